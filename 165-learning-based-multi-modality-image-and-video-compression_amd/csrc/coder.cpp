// Entropy coding side of the codec (host C++, include/cai_coder.h).
//
// (1) pmf -> 16-bit quantized CDF with frequency stealing, the table update()
//     builds for every entropy model (cpp_exts/ops/ops.cpp:40-109);
// (2) range-ANS with a 64-bit state emitting 32-bit words
//     (third_party/ryg_rans/rans64.h:59-142) and the escape scheme of
//     cpp_exts/rans/rans_interface.cpp:108-359: a symbol outside its CDF's
//     range codes the last CDF slot, then its overflow as 4-bit bypass
//     nibbles (count first, in 15-steps, then the nibbles low to high).
//
// Streams are byte-identical to the reference coder's for the same symbols,
// indexes and tables.  A stream is a serial state machine; parallelism is
// across streams (one per image) with host threads.  Nothing here touches the
// GPU: the symbols arrive from the quantize kernel (cai_quantize, SYMBOLS
// mode) already on the host.
#include "cai.h"
#include "cai_coder.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

thread_local std::string g_err;

int fail(int code, std::string msg) {
    g_err = std::move(msg);
    return code;
}

constexpr uint32_t kScaleBits = 16;                 // rans_interface.cpp:49
constexpr uint32_t kBypassBits = 4;                 // rans_interface.cpp:51
constexpr uint32_t kMaxBypass = (1u << kBypassBits) - 1;
constexpr uint64_t kRansL = 1ull << 31;             // rans64.h:59

// ---------------------------------------------------------------------------
// quantized CDF (ops.cpp:40-109), same integer arithmetic step by step
// ---------------------------------------------------------------------------
int quantized_cdf(const float* pmf, int n, int precision, int32_t* out, std::string& err) {
    for (int i = 0; i < n; ++i) {
        const float p = pmf[i];
        if (p < 0 || !std::isfinite(p)) {
            err = "Invalid `pmf`, non-finite or negative element found: " + std::to_string(p);
            return CAI_EINVAL;
        }
    }
    std::vector<uint32_t> cdf(n + 1);
    cdf[0] = 0;
    const float scale = (float)(1 << precision);
    for (int i = 0; i < n; ++i) cdf[i + 1] = (uint32_t)std::round(pmf[i] * scale);
    uint32_t total = 0;   // std::accumulate(..., 0): modular 32-bit sum
    for (uint32_t v : cdf) total += v;
    if (total == 0) {
        err = "Invalid `pmf`: at least one element must have a non-zero probability.";
        return CAI_EINVAL;
    }
    for (auto& v : cdf) v = (uint32_t)(((uint64_t)(1u << precision) * v) / total);
    for (size_t i = 1; i < cdf.size(); ++i) cdf[i] += cdf[i - 1];
    cdf.back() = 1u << precision;
    const int last = (int)cdf.size() - 1;
    for (int i = 0; i < last; ++i) {
        if (cdf[i] != cdf[i + 1]) continue;
        // a zero-frequency slot: steal one count from the smallest slot > 1
        uint32_t best_freq = ~0u;
        int best_steal = -1;
        for (int j = 0; j < last; ++j) {
            const uint32_t freq = cdf[j + 1] - cdf[j];
            if (freq > 1 && freq < best_freq) {
                best_freq = freq;
                best_steal = j;
            }
        }
        if (best_steal < 0) {
            err = "Invalid `pmf`: no frequency left to give every symbol a non-zero count";
            return CAI_EINVAL;
        }
        if (best_steal < i) {
            for (int j = best_steal + 1; j <= i; ++j) cdf[j]--;
        } else {
            for (int j = i + 1; j <= best_steal; ++j) cdf[j]++;
        }
    }
    for (int i = 0; i <= last; ++i) out[i] = (int32_t)cdf[i];
    return CAI_OK;
}

// run fn(i) for i in [0, n) on up to nthreads threads; first error wins
template <typename F>
int parallel_for(int64_t n, int nthreads, F fn) {
    if (n <= 0) return CAI_OK;
    nthreads = (int)std::max<int64_t>(1, std::min<int64_t>(nthreads <= 0 ? 1 : nthreads, n));
    std::atomic<int64_t> next{0};
    std::atomic<int> rc{CAI_OK};
    std::vector<std::string> errs(nthreads);
    auto body = [&](int w) {
        for (;;) {
            const int64_t i = next.fetch_add(1);
            if (i >= n || rc.load() != CAI_OK) return;
            const int r = fn(i, errs[w]);
            if (r != CAI_OK) {
                int expect = CAI_OK;
                if (rc.compare_exchange_strong(expect, r)) errs[w] = "item " + std::to_string(i) + ": " + errs[w];
                else errs[w].clear();
                return;
            }
        }
    };
    if (nthreads == 1) {
        body(0);
    } else {
        std::vector<std::thread> pool;
        for (int w = 0; w < nthreads; ++w) pool.emplace_back(body, w);
        for (auto& t : pool) t.join();
    }
    if (rc.load() != CAI_OK) {
        for (auto& e : errs)
            if (!e.empty()) return fail(rc.load(), e);
        return fail(rc.load(), "unknown error");
    }
    return CAI_OK;
}

// ---------------------------------------------------------------------------
// rANS
// ---------------------------------------------------------------------------
struct RansSym {
    uint16_t start, range;
    bool bypass;
};

int check_tables(const cai_rans_tables* t, std::string& err) {
    if (!t || !t->cdfs || !t->cdf_sizes || !t->offsets || t->n_cdfs <= 0 || t->cdf_stride < 2) {
        err = "invalid CDF tables";
        return CAI_EINVAL;
    }
    return CAI_OK;
}

// rans_interface.cpp:117-172: symbols -> (start, range) list, escapes as bypass nibbles
int push_symbols(std::vector<RansSym>& syms, const int32_t* symbols, const int32_t* indexes, int64_t n,
                 const cai_rans_tables* t, std::string& err) {
    for (int64_t i = 0; i < n; ++i) {
        const int32_t idx = indexes[i];
        if (idx < 0 || idx >= t->n_cdfs) {
            err = "cdf index " + std::to_string(idx) + " out of range [0, " + std::to_string(t->n_cdfs) + ")";
            return CAI_EINVAL;
        }
        const int32_t* cdf = t->cdfs + (int64_t)idx * t->cdf_stride;
        const int32_t max_value = t->cdf_sizes[idx] - 2;
        if (max_value < 0 || max_value + 1 >= t->cdf_stride) {
            err = "invalid cdf size for index " + std::to_string(idx);
            return CAI_EINVAL;
        }
        int32_t value = symbols[i] - t->offsets[idx];
        uint32_t raw_val = 0;
        if (value < 0) {
            raw_val = (uint32_t)(-2 * value - 1);
            value = max_value;
        } else if (value >= max_value) {
            raw_val = (uint32_t)(2 * (value - max_value));
            value = max_value;
        }
        const RansSym s{(uint16_t)cdf[value], (uint16_t)(cdf[value + 1] - cdf[value]), false};
        if (s.range == 0) {
            err = "zero-frequency symbol (cdf index " + std::to_string(idx) + ", slot " + std::to_string(value) + ")";
            return CAI_EINVAL;
        }
        syms.push_back(s);
        if (value == max_value) {
            int32_t n_bypass = 0;
            while (n_bypass < 8 && ((uint64_t)raw_val >> (n_bypass * kBypassBits)) != 0) ++n_bypass;
            int32_t val = n_bypass;
            while (val >= (int32_t)kMaxBypass) {
                syms.push_back({(uint16_t)kMaxBypass, (uint16_t)(kMaxBypass + 1), true});
                val -= kMaxBypass;
            }
            syms.push_back({(uint16_t)val, (uint16_t)(val + 1), true});
            for (int32_t j = 0; j < n_bypass; ++j) {
                const uint32_t nib = (raw_val >> (j * kBypassBits)) & kMaxBypass;
                syms.push_back({(uint16_t)nib, (uint16_t)(nib + 1), true});
            }
        }
    }
    return CAI_OK;
}

// words a flush of `count` symbols may emit: at most one renormalisation word
// per symbol (rans64.h:83-89) plus the 2-word final state
inline int64_t flush_words(int64_t count) { return count + 2; }

// rans_interface.cpp:175-200 (+ rans64.h:77-103): encode in reverse, write
// backwards; returns the byte count of the stream written to `out`
int flush_syms(const std::vector<RansSym>& syms, uint8_t* out, int64_t cap, int64_t* nbytes, std::string& err) {
    std::vector<uint32_t> buf((size_t)flush_words((int64_t)syms.size()));
    uint32_t* const end = buf.data() + buf.size();
    uint32_t* ptr = end;
    uint64_t x = kRansL;
    for (auto it = syms.rbegin(); it != syms.rend(); ++it) {
        const RansSym& s = *it;
        if (!s.bypass) {
            const uint64_t freq = s.range;
            const uint64_t x_max = ((kRansL >> kScaleBits) << 32) * freq;
            if (x >= x_max) {
                *--ptr = (uint32_t)x;
                x >>= 32;
            }
            x = ((x / freq) << kScaleBits) + (x % freq) + s.start;
        } else {
            const uint64_t freq = 1u << (16 - kBypassBits);
            const uint64_t x_max = ((kRansL >> 16) << 32) * freq;
            if (x >= x_max) {
                *--ptr = (uint32_t)x;
                x >>= 32;
            }
            x = (x << kBypassBits) | s.start;
        }
    }
    ptr -= 2;
    ptr[0] = (uint32_t)(x >> 0);
    ptr[1] = (uint32_t)(x >> 32);
    const int64_t bytes = (int64_t)(end - ptr) * 4;
    *nbytes = bytes;
    if (bytes > cap) {
        err = "output buffer of " + std::to_string(cap) + " bytes too small for " + std::to_string(bytes);
        return CAI_EWORKSPACE;
    }
    std::memcpy(out, ptr, (size_t)bytes);   // little-endian host: the reference's byte order
    return CAI_OK;
}

struct DecState {
    uint64_t x = 0;
    const uint32_t* ptr = nullptr;
    const uint32_t* end = nullptr;
};

inline bool refill(DecState& d) {
    if (d.x < kRansL) {
        if (d.ptr >= d.end) return false;
        d.x = (d.x << 32) | *d.ptr++;
    }
    return true;
}

int dec_init(DecState& d, const uint32_t* words, int64_t nwords, std::string& err) {
    if (nwords < 2) {
        err = "stream shorter than the 8-byte rANS state";
        return CAI_EINVAL;
    }
    d.x = (uint64_t)words[0] | ((uint64_t)words[1] << 32);
    d.ptr = words + 2;
    d.end = words + nwords;
    return CAI_OK;
}

// rans_interface.cpp:89-105
inline bool get_bits(DecState& d, uint32_t nbits, uint32_t& val) {
    val = (uint32_t)(d.x & ((1u << nbits) - 1));
    d.x >>= nbits;
    return refill(d);
}

// rans_interface.cpp:231-281 (one symbol per index)
int decode_symbols(DecState& d, const int32_t* indexes, int64_t n, const cai_rans_tables* t, int32_t* out,
                   std::string& err) {
    const char* trunc = "truncated or corrupt stream";
    for (int64_t i = 0; i < n; ++i) {
        const int32_t idx = indexes[i];
        if (idx < 0 || idx >= t->n_cdfs) {
            err = "cdf index " + std::to_string(idx) + " out of range";
            return CAI_EINVAL;
        }
        const int32_t* cdf = t->cdfs + (int64_t)idx * t->cdf_stride;
        const int32_t size = t->cdf_sizes[idx];
        const int32_t max_value = size - 2;
        if (max_value < 0 || max_value + 1 >= t->cdf_stride) {
            err = "invalid cdf size for index " + std::to_string(idx);
            return CAI_EINVAL;
        }
        const uint32_t cum = (uint32_t)(d.x & ((1u << kScaleBits) - 1));
        // first slot whose CDF value exceeds cum (the reference's linear
        // find_if; a binary search on the non-decreasing table finds the same)
        const int32_t* it = std::upper_bound(cdf, cdf + size, (int32_t)cum);
        const int32_t s = (int32_t)(it - cdf) - 1;
        if (s < 0 || s >= size - 1) {
            err = trunc;
            return CAI_EINVAL;
        }
        const uint64_t start = (uint32_t)cdf[s], freq = (uint32_t)(cdf[s + 1] - cdf[s]);
        d.x = freq * (d.x >> kScaleBits) + (d.x & ((1u << kScaleBits) - 1)) - start;
        if (!refill(d)) {
            err = trunc;
            return CAI_EINVAL;
        }
        int32_t value = s;
        if (value == max_value) {
            uint32_t val;
            if (!get_bits(d, kBypassBits, val)) {
                err = trunc;
                return CAI_EINVAL;
            }
            int32_t n_bypass = (int32_t)val;
            while (val == kMaxBypass) {
                if (!get_bits(d, kBypassBits, val)) {
                    err = trunc;
                    return CAI_EINVAL;
                }
                n_bypass += (int32_t)val;
            }
            if (n_bypass > 8) {
                err = trunc;
                return CAI_EINVAL;
            }
            uint32_t raw_val = 0;
            for (int32_t j = 0; j < n_bypass; ++j) {
                if (!get_bits(d, kBypassBits, val)) {
                    err = trunc;
                    return CAI_EINVAL;
                }
                raw_val |= val << (j * kBypassBits);
            }
            value = (int32_t)(raw_val >> 1);
            if (raw_val & 1)
                value = -value - 1;
            else
                value += max_value;
        }
        out[i] = value + t->offsets[idx];
    }
    return CAI_OK;
}

std::vector<uint32_t> to_words(const uint8_t* data, int64_t nbytes) {
    std::vector<uint32_t> w((size_t)(nbytes / 4));
    if (!w.empty()) std::memcpy(w.data(), data, w.size() * 4);
    return w;
}

int encode_one(const int32_t* symbols, const int32_t* indexes, int64_t n, const cai_rans_tables* t, uint8_t* out,
               int64_t cap, int64_t* nbytes, std::string& err) {
    std::vector<RansSym> syms;
    syms.reserve((size_t)n + 16);
    int rc = push_symbols(syms, symbols, indexes, n, t, err);
    if (rc) return rc;
    return flush_syms(syms, out, cap, nbytes, err);
}

int decode_one(const uint8_t* data, int64_t nbytes, const int32_t* indexes, int64_t n, const cai_rans_tables* t,
               int32_t* out, std::string& err) {
    if (nbytes < 0 || (nbytes & 3) != 0 || (nbytes > 0 && !data)) {
        err = "stream length must be a multiple of 4 bytes";
        return CAI_EINVAL;
    }
    const std::vector<uint32_t> words = to_words(data, nbytes);
    DecState d;
    int rc = dec_init(d, words.data(), (int64_t)words.size(), err);
    if (rc) return rc;
    return decode_symbols(d, indexes, n, t, out, err);
}

struct BufferedEncoder {
    std::vector<RansSym> syms;
};

struct StreamDecoder {
    std::vector<uint32_t> words;
    DecState st;
    bool ready = false;
};

}  // namespace

extern "C" {

const char* cai_coder_last_error(void) { return g_err.c_str(); }

int cai_coder_abi_count(void) { return 18; }

int cai_pmf_to_quantized_cdf(const float* pmf, int32_t n, int32_t precision, int32_t* cdf) {
    if (!pmf || !cdf || n < 1) return fail(CAI_EINVAL, "pmf_to_quantized_cdf: empty pmf");
    if (precision < 1 || precision > 24) return fail(CAI_EINVAL, "pmf_to_quantized_cdf: precision must be in [1, 24]");
    std::string err;
    const int rc = quantized_cdf(pmf, n, precision, cdf, err);
    return rc ? fail(rc, err) : CAI_OK;
}

int cai_pmf_to_quantized_cdf_rows(const float* pmf, int64_t pmf_stride, const int32_t* lengths, int32_t rows,
                                  int32_t precision, int32_t* cdf, int64_t cdf_stride, int32_t nthreads) {
    if (rows < 0 || (rows > 0 && (!pmf || !lengths || !cdf)))
        return fail(CAI_EINVAL, "pmf_to_quantized_cdf_rows: null pointer");
    if (precision < 1 || precision > 24)
        return fail(CAI_EINVAL, "pmf_to_quantized_cdf_rows: precision must be in [1, 24]");
    for (int32_t r = 0; r < rows; ++r)
        if (lengths[r] < 1 || lengths[r] > pmf_stride || lengths[r] + 1 > cdf_stride)
            return fail(CAI_EINVAL, "pmf_to_quantized_cdf_rows: row " + std::to_string(r) + " length " +
                                        std::to_string(lengths[r]) + " does not fit the strides");
    return parallel_for(rows, nthreads, [&](int64_t r, std::string& err) {
        return quantized_cdf(pmf + r * pmf_stride, lengths[r], precision, cdf + r * cdf_stride, err);
    });
}

int64_t cai_rans_max_bytes(int64_t n) {
    // per symbol: the symbol, <= 1 nibble-count escape (n_bypass <= 8 < 15)
    // and <= 8 nibbles
    return 4 * flush_words(10 * std::max<int64_t>(n, 0));
}

int cai_rans_encode(const int32_t* symbols, const int32_t* indexes, int64_t n, const cai_rans_tables* t,
                    uint8_t* out, int64_t cap, int64_t* nbytes) {
    std::string err;
    if (check_tables(t, err)) return fail(CAI_EINVAL, "rans_encode: " + err);
    if (n < 0 || (n > 0 && (!symbols || !indexes)) || !out || !nbytes)
        return fail(CAI_EINVAL, "rans_encode: null pointer");
    const int rc = encode_one(symbols, indexes, n, t, out, cap, nbytes, err);
    return rc ? fail(rc, "rans_encode: " + err) : CAI_OK;
}

int cai_rans_encode_batch(int32_t nstreams, const int32_t* symbols, const int32_t* indexes, const int64_t* sym_off,
                          const cai_rans_tables* t, uint8_t* out, const int64_t* out_off, int64_t* nbytes,
                          int32_t nthreads) {
    std::string err;
    if (check_tables(t, err)) return fail(CAI_EINVAL, "rans_encode_batch: " + err);
    if (nstreams < 0 || (nstreams > 0 && (!sym_off || !out_off || !nbytes || !out)))
        return fail(CAI_EINVAL, "rans_encode_batch: null pointer");
    for (int32_t s = 0; s < nstreams; ++s)
        if (sym_off[s + 1] < sym_off[s] || out_off[s + 1] < out_off[s])
            return fail(CAI_EINVAL, "rans_encode_batch: offsets must be non-decreasing");
    const int rc = parallel_for(nstreams, nthreads, [&](int64_t s, std::string& e) {
        return encode_one(symbols + sym_off[s], indexes + sym_off[s], sym_off[s + 1] - sym_off[s], t,
                          out + out_off[s], out_off[s + 1] - out_off[s], nbytes + s, e);
    });
    if (rc) g_err = "rans_encode_batch: " + g_err;
    return rc;
}

int cai_rans_decode(const uint8_t* data, int64_t nbytes, const int32_t* indexes, int64_t n, const cai_rans_tables* t,
                    int32_t* out) {
    std::string err;
    if (check_tables(t, err)) return fail(CAI_EINVAL, "rans_decode: " + err);
    if (n < 0 || (n > 0 && (!indexes || !out))) return fail(CAI_EINVAL, "rans_decode: null pointer");
    const int rc = decode_one(data, nbytes, indexes, n, t, out, err);
    return rc ? fail(rc, "rans_decode: " + err) : CAI_OK;
}

int cai_rans_decode_batch(int32_t nstreams, const uint8_t* data, const int64_t* data_off, const int64_t* nbytes,
                          const int32_t* indexes, const int64_t* sym_off, const cai_rans_tables* t, int32_t* out,
                          int32_t nthreads) {
    std::string err;
    if (check_tables(t, err)) return fail(CAI_EINVAL, "rans_decode_batch: " + err);
    if (nstreams < 0 || (nstreams > 0 && (!data || !data_off || !nbytes || !sym_off)))
        return fail(CAI_EINVAL, "rans_decode_batch: null pointer");
    for (int32_t s = 0; s < nstreams; ++s)
        if (sym_off[s + 1] < sym_off[s]) return fail(CAI_EINVAL, "rans_decode_batch: offsets must be non-decreasing");
    const int rc = parallel_for(nstreams, nthreads, [&](int64_t s, std::string& e) {
        return decode_one(data + data_off[s], nbytes[s], indexes + sym_off[s], sym_off[s + 1] - sym_off[s], t,
                          out + sym_off[s], e);
    });
    if (rc) g_err = "rans_decode_batch: " + g_err;
    return rc;
}

void* cai_rans_buffered_create(void) { return new (std::nothrow) BufferedEncoder(); }

void cai_rans_buffered_destroy(void* h) { delete reinterpret_cast<BufferedEncoder*>(h); }

int cai_rans_buffered_encode(void* h, const int32_t* symbols, const int32_t* indexes, int64_t n,
                             const cai_rans_tables* t) {
    std::string err;
    if (!h) return fail(CAI_EINVAL, "rans_buffered_encode: null handle");
    if (check_tables(t, err)) return fail(CAI_EINVAL, "rans_buffered_encode: " + err);
    if (n < 0 || (n > 0 && (!symbols || !indexes))) return fail(CAI_EINVAL, "rans_buffered_encode: null pointer");
    auto& syms = reinterpret_cast<BufferedEncoder*>(h)->syms;
    const size_t before = syms.size();
    const int rc = push_symbols(syms, symbols, indexes, n, t, err);
    if (rc) {
        syms.resize(before);   // a rejected call leaves the buffer as it was
        return fail(rc, "rans_buffered_encode: " + err);
    }
    return CAI_OK;
}

int64_t cai_rans_buffered_max_bytes(void* h) {
    if (!h) return -1;
    return 4 * flush_words((int64_t)reinterpret_cast<BufferedEncoder*>(h)->syms.size());
}

int cai_rans_buffered_flush(void* h, uint8_t* out, int64_t cap, int64_t* nbytes) {
    if (!h || !out || !nbytes) return fail(CAI_EINVAL, "rans_buffered_flush: null pointer");
    auto& syms = reinterpret_cast<BufferedEncoder*>(h)->syms;
    std::string err;
    const int rc = flush_syms(syms, out, cap, nbytes, err);
    if (rc) return fail(rc, "rans_buffered_flush: " + err);
    syms.clear();
    return CAI_OK;
}

void* cai_rans_decoder_create(void) { return new (std::nothrow) StreamDecoder(); }

void cai_rans_decoder_destroy(void* h) { delete reinterpret_cast<StreamDecoder*>(h); }

int cai_rans_decoder_set_stream(void* h, const uint8_t* data, int64_t nbytes) {
    if (!h) return fail(CAI_EINVAL, "rans_decoder_set_stream: null handle");
    if (nbytes < 0 || (nbytes & 3) != 0 || (nbytes > 0 && !data))
        return fail(CAI_EINVAL, "rans_decoder_set_stream: stream length must be a multiple of 4 bytes");
    auto* d = reinterpret_cast<StreamDecoder*>(h);
    d->words = to_words(data, nbytes);
    d->ready = false;
    std::string err;
    const int rc = dec_init(d->st, d->words.data(), (int64_t)d->words.size(), err);
    if (rc) return fail(rc, "rans_decoder_set_stream: " + err);
    d->ready = true;
    return CAI_OK;
}

int cai_rans_decoder_decode_stream(void* h, const int32_t* indexes, int64_t n, const cai_rans_tables* t,
                                   int32_t* out) {
    std::string err;
    if (!h) return fail(CAI_EINVAL, "rans_decoder_decode_stream: null handle");
    auto* d = reinterpret_cast<StreamDecoder*>(h);
    if (!d->ready) return fail(CAI_EINVAL, "rans_decoder_decode_stream: set_stream() first");
    if (check_tables(t, err)) return fail(CAI_EINVAL, "rans_decoder_decode_stream: " + err);
    if (n < 0 || (n > 0 && (!indexes || !out))) return fail(CAI_EINVAL, "rans_decoder_decode_stream: null pointer");
    const int rc = decode_symbols(d->st, indexes, n, t, out, err);
    return rc ? fail(rc, "rans_decoder_decode_stream: " + err) : CAI_OK;
}

}  // extern "C"
