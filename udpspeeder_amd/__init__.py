"""udpspeeder_amd -- MI355X-native Reed-Solomon erasure coding for UDPspeeder.

The drop-in for UDPspeeder's rs_encode2 / rs_decode2 hot path (lib/rs.h) is
librsmi.so (HIP kernels for gfx950 + C ABI, udpspeeder_amd/csrc).  This
package is its Python surface; see ``udpspeeder_amd.rs``.
"""
from ._lib import LIB_PATH, RsmiError, lib  # noqa: F401
from .fec_param import rs_from_str, rs_to_str  # noqa: F401
from .rs import (bitslice_source, code_encoder, precompile_code, wait_code,  # noqa: F401
                 decode, decode_host, decode_matrix, reference_rows, ref_slot_map, enc_matrix, encode,  # noqa: F401
                 encode_host, encode_ragged, fec_decode, fec_encode, fec_free, fec_new,
                 fill_data, get_code, get_k, get_n, make_groups, prepare_code, reserve,
                 rs_decode, rs_decode2, rs_encode, rs_encode2, version)

__all__ = [
    "rs_encode2", "rs_decode2", "rs_encode", "rs_decode", "fec_new", "fec_free", "fec_encode",
    "fec_decode", "get_k", "get_n", "get_code", "encode", "decode", "encode_ragged",
    "make_groups", "fill_data", "enc_matrix", "decode_matrix", "prepare_code", "reserve",
    "encode_host", "decode_host", "wait_code", "precompile_code", "code_encoder",
    "bitslice_source", "reference_rows", "ref_slot_map", "rs_from_str", "rs_to_str", "lib", "RsmiError", "LIB_PATH",
]
