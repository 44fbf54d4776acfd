/*
 * tbe_tools.h -- test / benchmark utilities exported by libtbe.so.
 *
 * Not a reference interface (the reference has no trace generator):
 * these helpers build synthetic request batches directly in device memory so that
 * benchmarks keep PCIe out of the timed region.  Streams are bit-identical to
 * oracle/trace.py and oracle/tb_ref.c.
 */
#ifndef TBE_TOOLS_H_
#define TBE_TOOLS_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Batch of n requests with global request counter g = g0 + i:
 *   keys[i]    = ((mix64(seed + g*GAMMA) >> 32) * n_keys) >> 32
 *   permits[i] = p_lo if p_lo == p_hi, else uniform on {p_lo..p_hi} from stream 0xA5..A5
 *   ts[i]      = ts0_us + (i * interval_us) / n                       (non-decreasing)
 * Enqueued on `stream` (hipStream_t or NULL).  Returns 0 on success. */
int tbe_gen_batch_device(uint64_t seed, uint64_t n_keys, uint64_t g0, uint64_t n, int32_t p_lo,
                         int32_t p_hi, int64_t ts0_us, int64_t interval_us, uint64_t *d_keys,
                         int32_t *d_permits, int64_t *d_ts, void *stream);

/* n keys of a bounded Zipf(s) stream over [0, n_items) (rank 1 hottest; ranks mapped to
 * keys by the fixed bijection of workloads.py), draws g0 .. g0+n-1, by rejection-
 * inversion.  s > 0, s != 1.  Enqueued on `stream`; returns 0 on success. */
int tbe_gen_zipf_keys_device(uint64_t seed, uint64_t n_items, double s, uint64_t g0, uint64_t n,
                             uint64_t *d_keys, void *stream);

/* out[i] = the engine's device round trip of in[i] through Lua tostring ("%.14g") and
 * C# double.Parse (csrc/tbe_numfmt.hpp; A:270 -> A:442), for parity tests of the gfx950
 * build.  Enqueued on `stream`; returns 0 on success. */
int tbe_numfmt_device(const double *d_in, double *d_out, uint64_t n, void *stream);

/* Synthetic string keys (string-directory tests and benchmark): key text i = prefix +
 * decimal(keys[i]).  lens[i] = prefix_len + its digit count (prefix_len <= 32); after the
 * caller's scan into n + 1 offsets, the text of key i fills bytes[offs[i], offs[i+1])
 * (digits right-aligned, zero-padded on the left when the span is longer).  Enqueued on
 * `stream`; returns 0 on success. */
int tbe_key_text_lengths_device(const uint64_t *d_keys, uint64_t n, uint32_t prefix_len, uint64_t *d_lens,
                                void *stream);
int tbe_key_text_device(const uint64_t *d_keys, uint64_t n, const char *prefix, uint32_t prefix_len,
                        const uint64_t *d_offs, uint8_t *d_bytes, void *stream);

/* Profiling marker: enqueues one empty dispatch named k_mark<tag> (tag 1 to 4), so that a
 * rocprofv3 trace can keep exactly the dispatches enqueued between two markers: 1 and 2
 * bracket the benchmark's timed batches, 3 and 4 the serial replay of them that the bench
 * line's roofline times (tools/prof_window.py).  Returns 0 on success. */
int tbe_mark_device(uint32_t tag, void *stream);

/* HBM-counter calibration (k_calib<mode>): reads or writes a known byte count with one
 * access shape -- 0/1/2 streaming reads of 16/8/4 B per lane, 3/4/5 gathers of 16/8/4 B
 * per lane at hashed 128-byte lines, 6/7 streaming writes of 16/4 B per lane, 8/9
 * scatters of 16/1 B per lane -- over n elements of the `bytes`-byte buffer d_buf
 * (bytes a multiple of 128; streams need n * width <= bytes).  d_sink: one u64 of device
 * memory.  Returns 0 on success. */
int tbe_calib_device(uint32_t mode, uint8_t *d_buf, uint64_t bytes, uint64_t n, uint64_t *d_sink, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* TBE_TOOLS_H_ */
