/*
 * libcai_coder -- C ABI of the entropy-coding side of the codec (host code).
 *
 * the quantized-CDF tables built by update() and the
 * rANS bitstream coder used by compress() / decompress().  The reference runs
 * these on the CPU as pybind11 modules; they stay host code here (a serial
 * rANS state machine per stream), but streams are independent, so the batch
 * entry points code one stream per image across host threads.
 *
 * Reference interfaces replaced (paths relative to /root/reference/CompressAI):
 *   compressai._CXX.pmf_to_quantized_cdf ..... compressai/cpp_exts/ops/ops.cpp:40-109,116-117
 *   EntropyModel._pmf_to_cdf (row loop) ...... compressai/entropy_models/entropy_models.py:206-214
 *   compressai.ans.RansEncoder ............... compressai/cpp_exts/rans/rans_interface.cpp:202-213,371-373
 *   compressai.ans.BufferedRansEncoder ....... rans_interface.cpp:108-200,366-369
 *   compressai.ans.RansDecoder ............... rans_interface.cpp:215-359,375-380
 *   rANS primitives .......................... third_party/ryg_rans/rans64.h:59-142 (64-bit state, 32-bit words)
 *
 * Conventions: plain host pointers; return 0 (CAI_OK) or a CAI_E* code from
 * cai.h with a thread-local message in cai_coder_last_error().  Arguments the
 * reference only asserts on (asserts compiled out with NDEBUG, i.e. undefined
 * behaviour there: bad CDF index, zero-frequency symbol, truncated stream) are
 * rejected with CAI_EINVAL here.  A stream's bytes are the reference's:
 * little-endian 32-bit words, the final encoder state (2 words) first.
 */
#ifndef CAI_CODER_H
#define CAI_CODER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

const char* cai_coder_last_error(void);
/* number of entry points exported below (checked by the loader test) */
int cai_coder_abi_count(void);

/* ---- quantized CDFs (ops.cpp:40-109) ----------------------------------- */
/* cdf[0..n] (n + 1 entries) from pmf[0..n-1]; 1 <= precision <= 24.  A
 * negative or non-finite element, or an all-zero pmf, is CAI_EINVAL
 * (std::domain_error -> ValueError in the reference). */
int cai_pmf_to_quantized_cdf(const float* pmf, int32_t n, int32_t precision, int32_t* cdf);

/* _pmf_to_cdf over a table: row r of pmf (row stride pmf_stride elements)
 * holds lengths[r] probabilities (pmf_length + the tail mass); its CDF
 * (lengths[r] + 1 entries) goes to cdf + r * cdf_stride, the rest of the row
 * is left untouched.  Rows are independent (up to nthreads host threads). */
int cai_pmf_to_quantized_cdf_rows(const float* pmf, int64_t pmf_stride, const int32_t* lengths, int32_t rows,
                                  int32_t precision, int32_t* cdf, int64_t cdf_stride, int32_t nthreads);

/* ---- rANS (rans_interface.cpp, precision 16, 4-bit bypass escapes) ------ */
typedef struct cai_rans_tables {
    const int32_t* cdfs;        /* [n_cdfs][cdf_stride] quantized CDFs           */
    int64_t cdf_stride;
    const int32_t* cdf_sizes;   /* [n_cdfs] valid entries per CDF (pmf_length+2) */
    const int32_t* offsets;     /* [n_cdfs] symbol offset per CDF                */
    int32_t n_cdfs;
} cai_rans_tables;

/* upper bound of the encoded size of n symbols (bytes) */
int64_t cai_rans_max_bytes(int64_t n);

/* RansEncoder.encode_with_indexes: one stream of n symbols.  Writes *nbytes
 * bytes to out (cap >= cai_rans_max_bytes(n) always suffices). */
int cai_rans_encode(const int32_t* symbols, const int32_t* indexes, int64_t n, const cai_rans_tables* t,
                    uint8_t* out, int64_t cap, int64_t* nbytes);

/* nstreams independent streams: stream s codes symbols/indexes
 * [sym_off[s], sym_off[s+1]) into out + out_off[s] (capacity
 * out_off[s+1] - out_off[s]); its size goes to nbytes[s]. */
int cai_rans_encode_batch(int32_t nstreams, const int32_t* symbols, const int32_t* indexes, const int64_t* sym_off,
                          const cai_rans_tables* t, uint8_t* out, const int64_t* out_off, int64_t* nbytes,
                          int32_t nthreads);

/* RansDecoder.decode_with_indexes: n symbols from one stream. */
int cai_rans_decode(const uint8_t* data, int64_t nbytes, const int32_t* indexes, int64_t n, const cai_rans_tables* t,
                    int32_t* out);

/* stream s: data + data_off[s] (nbytes[s] bytes) -> out[sym_off[s] .. sym_off[s+1]) */
int cai_rans_decode_batch(int32_t nstreams, const uint8_t* data, const int64_t* data_off, const int64_t* nbytes,
                          const int32_t* indexes, const int64_t* sym_off, const cai_rans_tables* t, int32_t* out,
                          int32_t nthreads);

/* BufferedRansEncoder: encode() any number of times, then flush() the whole
 * stream (the autoregressive models code one latent pixel at a time,
 * google.py:565-608). */
void* cai_rans_buffered_create(void);
void cai_rans_buffered_destroy(void* h);
int cai_rans_buffered_encode(void* h, const int32_t* symbols, const int32_t* indexes, int64_t n,
                             const cai_rans_tables* t);
/* bytes the next flush() may need */
int64_t cai_rans_buffered_max_bytes(void* h);
/* writes the stream and empties the buffer */
int cai_rans_buffered_flush(void* h, uint8_t* out, int64_t cap, int64_t* nbytes);

/* RansDecoder.set_stream / decode_stream: a decoder that keeps its state
 * between calls (the stream is copied). */
void* cai_rans_decoder_create(void);
void cai_rans_decoder_destroy(void* h);
int cai_rans_decoder_set_stream(void* h, const uint8_t* data, int64_t nbytes);
int cai_rans_decoder_decode_stream(void* h, const int32_t* indexes, int64_t n, const cai_rans_tables* t,
                                   int32_t* out);

#ifdef __cplusplus
}
#endif
#endif /* CAI_CODER_H */
