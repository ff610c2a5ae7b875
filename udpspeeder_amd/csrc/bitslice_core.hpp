// bitslice_core.hpp -- the in-register 8x8 bit transpose used by the
// bit-sliced encoders (gen/bitslice_codes.inc).  Per byte lane b of eight
// dwords w[0..7], bit t of byte b of w[q] moves to bit q of byte b of w[t]:
// after the call w[t] is bit-plane t (bit t of 32 byte positions).  The three
// block-swap stages commute, so the routine is its own inverse.
// Included by bitslice.hip (device) and by the CPU test harness (host).
#pragma once

template <int D, uint32_t MASK>
__host__ __device__ __forceinline__ void bs_swap(uint32_t &a, uint32_t &b) {
    // a keeps its low field, takes b's low field into its high field;
    // b keeps its high field, takes a's high field into its low field.
    const uint32_t na = (a & MASK) | ((b << D) & ~MASK);
    const uint32_t nb = ((a >> D) & MASK) | (b & ~MASK);
    a = na;
    b = nb;
}

__host__ __device__ __forceinline__ void bs_transpose8(uint32_t (&w)[8]) {
    bs_swap<4, 0x0F0F0F0Fu>(w[0], w[4]);
    bs_swap<4, 0x0F0F0F0Fu>(w[1], w[5]);
    bs_swap<4, 0x0F0F0F0Fu>(w[2], w[6]);
    bs_swap<4, 0x0F0F0F0Fu>(w[3], w[7]);
    bs_swap<2, 0x33333333u>(w[0], w[2]);
    bs_swap<2, 0x33333333u>(w[1], w[3]);
    bs_swap<2, 0x33333333u>(w[4], w[6]);
    bs_swap<2, 0x33333333u>(w[5], w[7]);
    bs_swap<1, 0x55555555u>(w[0], w[1]);
    bs_swap<1, 0x55555555u>(w[2], w[3]);
    bs_swap<1, 0x55555555u>(w[4], w[5]);
    bs_swap<1, 0x55555555u>(w[6], w[7]);
}
