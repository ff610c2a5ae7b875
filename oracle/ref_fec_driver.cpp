// TEST INFRASTRUCTURE ONLY -- never shipped, never on the product path.
//
// Thin extern "C" driver around the REAL reference FEC managers
// (/root/reference/fec_manager.cpp, compiled unmodified from where it lies by
// oracle/Makefile with the reference sources it links against).  Used to
// generate tests/golden/fec_*.npz and to pin oracle/fec_frame.py.
//
//   fec_encode_manager_t::input / output   fec_manager.cpp:206-460
//   fec_decode_manager_t::input / output   fec_manager.cpp:469-797
//   g_fec_par (fec_parameter_t)            fec_manager.h:26-180, misc.cpp:587
//
// The encoder's first sequence number is drawn by the reference
// (get_fake_random_number, fec_manager.h:327); callers read it back from the
// first packet header.
//
// Managers are constructed in zeroed memory.  Their constructors leave the
// big buffers uninitialised (blob_encode_t::input_buf, fec_manager.h:257;
// the decoder's ring), and the encoder sends bytes of blob_encode_t's buffer
// past the blob's end (blob_encode_t::output, fec_manager.cpp:67-75): zeroed
// memory (what a fresh process's mmap-backed allocation of these ~2 MB
// objects holds) makes those bytes a function of the connection's history
// alone, so the fixtures are deterministic.
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>

#include "common.h"
#include "fec_manager.h"
#include "log.h"

static void empty_cb(struct ev_loop *, struct ev_timer *, int) {}

template <class T>
static T *new_zeroed() {
    void *mem = std::calloc(1, sizeof(T));
    return mem ? new (mem) T() : nullptr;
}

template <class T>
static void free_zeroed(T *p) {
    if (!p) return;
    p->~T();
    std::free(p);
}


extern "C" {

// -f rs_str, --mode, --mtu, --queue-len (misc.cpp:587, 265-294); returns
// rs_from_str's result.  Also silences the reference's logging.
int ref_fec_config(const char *rs_str, int mode, int mtu, int queue_len) {
    log_level = log_fatal;
    g_fec_par.mode = mode;
    g_fec_par.mtu = mtu;
    g_fec_par.queue_len = queue_len;
    int rc = g_fec_par.rs_from_str((char *)rs_str);
    g_fec_par.version++;
    return rc;
}

// fec_parameter_t::rs_from_str (fec_manager.h:40-136) on a fresh table:
// returns its result (0 or -1), the table size in *cnt and y of x = 1..cnt.
int ref_rs_table(const char *rs_str, int *cnt, int *ys) {
    log_level = log_fatal;
    fec_parameter_t *p = new_zeroed<fec_parameter_t>();
    std::string tmp(rs_str);
    int rc = p->rs_from_str((char *)tmp.c_str());
    *cnt = rc == 0 ? p->rs_cnt : 0;
    for (int i = 0; i < *cnt; ++i) ys[i] = p->rs_par[i].y;
    free_zeroed(p);
    return rc;
}

void *ref_fenc_new() {
    fec_encode_manager_t *m = new_zeroed<fec_encode_manager_t>();
    m->set_loop_and_cb(ev_default_loop(0), empty_cb);  // as misc.cpp:398 (timer never runs)
    return m;
}

void ref_fenc_free(void *h) { free_zeroed((fec_encode_manager_t *)h); }

// Feed events to input(); after each, collect output().  len[i] >= 0: packet
// at buf + off[i]; len[i] < 0: input(0, 0).  Emitted packets are appended to
// out (out_len[j] bytes each, at out_pos[j]) with out_event[j] = i.  Returns
// the number of packets emitted, or -1 if out/max_out overflowed.
int64_t ref_fenc_run(void *h, int64_t n, const int32_t *len, const uint64_t *off,
                     const uint8_t *buf, int32_t *ret, uint8_t *out, int64_t out_cap,
                     int64_t *out_pos, int32_t *out_len, int32_t *out_event, int64_t max_out) {
    fec_encode_manager_t *m = (fec_encode_manager_t *)h;
    int64_t np = 0, pos = 0;
    for (int64_t i = 0; i < n; ++i) {
        int r = len[i] >= 0 ? m->input((char *)(buf + off[i]), len[i]) : m->input(0, 0);
        if (ret) ret[i] = r;
        int on;
        char **arr;
        int *ol;
        m->output(on, arr, ol);
        for (int j = 0; j < on; ++j) {
            if (np >= max_out || pos + ol[j] > out_cap) return -1;
            std::memcpy(out + pos, arr[j], ol[j]);
            out_pos[np] = pos;
            out_len[np] = ol[j];
            out_event[np] = (int32_t)i;
            pos += ol[j];
            ++np;
        }
    }
    return np;
}

void *ref_fdec_new() { return new_zeroed<fec_decode_manager_t>(); }

void ref_fdec_free(void *h) { free_zeroed((fec_decode_manager_t *)h); }

// Feed packets to fec_decode_manager_t::input (each copied into a buf_len
// buffer first, as the receive path's buffers are); after each, collect
// output().  Same output convention as ref_fenc_run.
int64_t ref_fdec_run(void *h, int64_t n, const int32_t *len, const uint64_t *off,
                     const uint8_t *buf, int32_t *ret, uint8_t *out, int64_t out_cap,
                     int64_t *out_pos, int32_t *out_len, int32_t *out_event, int64_t max_out) {
    fec_decode_manager_t *m = (fec_decode_manager_t *)h;
    static char tmp[buf_len];
    int64_t np = 0, pos = 0;
    for (int64_t i = 0; i < n; ++i) {
        int l = len[i];
        if (l < 0 || l + 100 >= buf_len) {
            if (ret) ret[i] = -2;  // the reference asserts len + 100 < buf_len
            continue;
        }
        std::memcpy(tmp, buf + off[i], l);
        int r = m->input(tmp, l);
        if (ret) ret[i] = r;
        int on;
        char **arr;
        int *ol;
        m->output(on, arr, ol);
        for (int j = 0; j < on; ++j) {
            if (np >= max_out || pos + ol[j] > out_cap) return -1;
            std::memcpy(out + pos, arr[j], ol[j]);
            out_pos[np] = pos;
            out_len[np] = ol[j];
            out_event[np] = (int32_t)i;
            pos += ol[j];
            ++np;
        }
    }
    return np;
}

}  // extern "C"
