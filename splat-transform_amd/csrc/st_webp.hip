// st_webp.hip -- WebP lossless (VP8L) encode and CRC-32 on the device (SURVEY.md
// 8f ranks 1 and 3).
//
// Replaces WebPEncodeLosslessRGBA (lib/webp_encode.c:19-29 via utils/webp.ts:19-41,
// used by write-sog.ts:120-140) and Crc (serialize/crc.ts:1-28, used by
// serialize/zip-writer.ts).  Parity is at the decoded-RGBA level:
// the stream is a valid VP8L image that decodes to exactly the input pixels.
//
// Encoding (all HBM-bound byte work; one image = W x H RGBA8, <= 16384^2):
//   k_vp8l_predict  one workgroup per 16 x 16 block: the 14 VP8L predictors are
//                   scored on the block (sum of |signed residual|), the cheapest
//                   wins, residuals (pixel - prediction per channel, mod 256) are
//                   written as ARGB words                  read 4 B (+ neighbours), write 4 B
//   k_vp8l_runs     per 4,096-pixel group: runs of >= 3 residuals equal to their left
//                   neighbour become one LZ77 copy (distance code 2: the pixel to the
//                   left; length <= 4,096), tokens: literal / copy length / covered
//   k_cc_tab        colour cache (RFC 9649 5.2.2), all candidate sizes 2^4..2^10 at once: per
//                   4,096-pixel group, the last colour written to each cache slot  read 4 B
//   k_cc_scan1/2    the cache state at each group's start: per slot, the last group before it
//                   that wrote the slot (a carry scan over chunks of 64 groups, then over chunks)
//   k_cc_walk       per group one wave whose lanes 0..6 each replay one cache size over the
//                   group's pixels in order from that state (LDS table; reads and writes issued
//                   back to back, the compares after): a pixel hits when the last earlier pixel
//                   with its index has its colour                      read 4 B, write 1 B
//   k_cc_survey     per size, the literals' hits as histograms: the host picks the size
//                   (vp8l::choose_cache_bits) and k_vp8l_hist redoes the histograms with it
//   k_vp8l_hist     symbol histograms (literal channels, length prefixes, cache indices,
//                   distance; LDS-private, one flush per group)        read 4 + 2 + 1 B
//   host            canonical length-limited prefix codes + header bits (st_vp8l.cpp)
//   k_vp8l_bits     bits per 4,096-pixel group (table lookups in LDS)     read 4 B
//   k_vp8l_scan     exclusive bit offsets of the groups (one workgroup) + RIFF sizes
//   k_vp8l_emit     each group assembles its bit run in LDS (atomicOr at the run's
//                   own bit alignment) and stores whole words; the two edge words
//                   it shares with its neighbours are OR-ed in        read 4 B, write ~bits/8
// CRC-32: each thread takes the zlib CRC of a 2 KiB span (slicing-by-8) and shifts it to the end
// of the buffer (multiplication by x^(8m) mod P, zlib's crc32_combine identity);
// the XOR of all shifted CRCs is the CRC of the buffer.
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <thread>

#include "st_internal.h"
#include "st_vp8l.h"
#include "st_webp.h"

namespace st {
namespace {

constexpr int PB = 1 << vp8l::kPredBits;  // predictor block edge (16)
constexpr int EMIT_PP = 16;               // pixels per thread in the bit kernels
constexpr int EMIT_PIX = 256 * EMIT_PP;   // pixels per group
constexpr int EMIT_WORDS = EMIT_PIX * 60 / 32 + 2;

// prefix-code groups (the entropy image): blocks of 2^GROUP_BITS pixels where a literal carries
// a non-zero alpha residual (the edge of the zero padding after the last splat) take group 1,
// so every other pixel's alpha stays a one-symbol (zero-bit) code
constexpr int GROUP_BITS = 5;
constexpr int CODE_GROUPS = 2;

// tokens: a literal pixel, the start of an LZ77 copy (its length), or a pixel a copy covers
constexpr uint16_t TOK_LIT = 0, TOK_COVERED = 0xffffu;
constexpr uint32_t RUN_MIN = 3;                // shortest run coded as a copy
constexpr uint32_t DIST_LEFT_PREFIX = 1;       // distance code 2 = (1, 0): the pixel to the left

// LZ77 prefix coding of a length or distance value v >= 1 (RFC 9649 5.2.2): prefix code and
// extra bits
__device__ inline void prefix_of(uint32_t v, uint32_t &prefix, uint32_t &nextra, uint32_t &extra) {
    if (v <= 4) {
        prefix = v - 1;
        nextra = 0;
        extra = 0;
        return;
    }
    const uint32_t d = v - 1;
    const uint32_t hb = 31 - __builtin_clz(d);
    const uint32_t second = (d >> (hb - 1)) & 1u;
    nextra = hb - 1;
    extra = d & ((1u << nextra) - 1);
    prefix = 2 * hb + second;
}

// RGBA8 bytes (little endian word R | G<<8 | B<<16 | A<<24) -> VP8L ARGB word
__device__ inline uint32_t to_argb(uint32_t v) { return (v & 0xff00ff00u) | ((v & 0xffu) << 16) | ((v >> 16) & 0xffu); }

__device__ inline uint32_t ch(uint32_t v, int c) { return (v >> (8 * c)) & 0xffu; }

__device__ inline uint32_t avg2(uint32_t a, uint32_t b) { return (((a ^ b) & 0xfefefefeu) >> 1) + (a & b); }

__device__ inline uint32_t clamp_add_sub_full(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        int v = (int)ch(a, k) + (int)ch(b, k) - (int)ch(c, k);
        v = v < 0 ? 0 : (v > 255 ? 255 : v);
        r |= (uint32_t)v << (8 * k);
    }
    return r;
}

__device__ inline uint32_t clamp_add_sub_half(uint32_t a, uint32_t b) {
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int x = (int)ch(a, k), y = (int)ch(b, k);
        int v = x + (x - y) / 2;  // C division: truncation toward zero, as the format defines
        v = v < 0 ? 0 : (v > 255 ? 255 : v);
        r |= (uint32_t)v << (8 * k);
    }
    return r;
}

// Select(L, T, TL): L when its Manhattan distance to L + T - TL is strictly smaller
__device__ inline uint32_t select_pred(uint32_t L, uint32_t T, uint32_t TL) {
    int pl = 0, pt = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int l = (int)ch(L, k), t = (int)ch(T, k), tl = (int)ch(TL, k);
        pl += abs(t - tl);  // |(L + T - TL) - L|
        pt += abs(l - tl);  // |(L + T - TL) - T|
    }
    return (pl < pt) ? L : T;
}

__device__ inline uint32_t predict(int m, uint32_t L, uint32_t T, uint32_t TL, uint32_t TR) {
    switch (m) {
        case 0: return 0xff000000u;
        case 1: return L;
        case 2: return T;
        case 3: return TR;
        case 4: return TL;
        case 5: return avg2(avg2(L, TR), T);
        case 6: return avg2(L, TL);
        case 7: return avg2(L, T);
        case 8: return avg2(TL, T);
        case 9: return avg2(T, TR);
        case 10: return avg2(avg2(L, TL), avg2(T, TR));
        case 11: return select_pred(L, T, TL);
        case 12: return clamp_add_sub_full(L, T, TL);
        default: return clamp_add_sub_half(avg2(L, T), TL);
    }
}

// per-channel (a - b) mod 256
__device__ inline uint32_t sub_pixels(uint32_t a, uint32_t b) {
    const uint32_t ag = (a | 0x00ff00ffu) - (b & 0xff00ff00u);
    const uint32_t rb = (a | 0xff00ff00u) - (b & 0x00ff00ffu);
    return (ag & 0xff00ff00u) | (rb & 0x00ff00ffu);
}

__device__ inline uint32_t residual_cost(uint32_t r) {
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t v = ch(r, k);
        s += v < 128 ? v : 256 - v;
    }
    return s;
}

__global__ __launch_bounds__(256) void k_vp8l_predict(const uint8_t *__restrict__ rgba, int w, int h, int stride,
                                                      int bw, uint8_t *__restrict__ modes,
                                                      uint32_t *__restrict__ resid, int force_mode) {
    __shared__ uint32_t part[4][14];
    __shared__ uint32_t alpha_any;
    if (threadIdx.x == 0) alpha_any = 0;
    __syncthreads();
    const int bx = blockIdx.x % bw, by = blockIdx.x / bw;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int x = bx * PB + (t & (PB - 1)), y = by * PB + (t >> vp8l::kPredBits);
    const bool valid = x < w && y < h;
    auto px = [&](int xx, int yy) -> uint32_t {
        return to_argb(*(const uint32_t *)(rgba + (size_t)yy * stride + (size_t)xx * 4));
    };
    uint32_t C = 0, L = 0, T = 0, TL = 0, TR = 0;
    if (valid) {
        C = px(x, y);
        if (x > 0) L = px(x - 1, y);
        if (y > 0) {
            T = px(x, y - 1);
            if (x > 0) TL = px(x - 1, y - 1);
            // the rightmost column's top-right is the leftmost pixel of the current row
            TR = (x + 1 < w) ? px(x + 1, y - 1) : px(0, y);
        }
    }
    if (__ballot(valid && (C >> 24) != 0xffu) && lane == 0) atomicOr(&alpha_any, 1u);
    const bool interior = valid && x > 0 && y > 0 && force_mode < 0;
    uint32_t cost[14];
#pragma unroll
    for (int m = 0; m < 14; ++m) cost[m] = interior ? residual_cost(sub_pixels(C, predict(m, L, T, TL, TR))) : 0u;
#pragma unroll
    for (int m = 0; m < 14; ++m)
        for (int o = 32; o > 0; o >>= 1) cost[m] += __shfl_xor(cost[m], o, 64);
    if (lane == 0)
#pragma unroll
        for (int m = 0; m < 14; ++m) part[wv][m] = cost[m];
    __syncthreads();
    __shared__ int best_s;
    if (t == 0) {
        int best = 0;  // the lowest mode among equal costs
        uint32_t bc = ~0u;
        for (int m = 0; m < 14; ++m) {
            const uint32_t s = part[0][m] + part[1][m] + part[2][m] + part[3][m];
            if (s < bc) {
                bc = s;
                best = m;
            }
        }
        if (force_mode >= 0) best = force_mode;
        best_s = best;
        // bit 7: some pixel of the block has alpha != 255 (the header's alpha hint)
        modes[blockIdx.x] = (uint8_t)(best | (alpha_any ? 0x80 : 0));
    }
    __syncthreads();
    if (!valid) return;
    uint32_t pred;
    if (y == 0)
        pred = (x == 0) ? 0xff000000u : L;
    else if (x == 0)
        pred = T;
    else
        pred = predict(best_s, L, T, TL, TR);
    resid[(size_t)y * w + x] = sub_pixels(C, pred);
}

// symbol histograms in the vp8l::kOff* layout
// group of pixel p (the block's flag), from its row and column
__device__ inline uint32_t group_of(const uint8_t *gflag, uint32_t p, int w, int gw) {
    const uint32_t y = p / (uint32_t)w, x = p - y * (uint32_t)w;
    return gflag[(y >> GROUP_BITS) * (uint32_t)gw + (x >> GROUP_BITS)];
}

// symbol histograms per prefix-code group (CODE_GROUPS x kTabSize, the vp8l::kOff* layout) and,
// with raw, the histogram of the pixels themselves as predictor 0 leaves them (pixel - 0xff000000):
// the host's per-image choice between the chosen predictors and none
// colour-cache index of an ARGB word in a 2^bits-entry cache
__device__ inline uint32_t cc_index(uint32_t argb, int bits) { return (argb * vp8l::kCacheMul) >> (32 - bits); }
// a literal coded as a cache index (cb: the image's cache bits, 0 = no cache)
__device__ inline bool cc_hit(const uint8_t *hits, uint64_t p, int cb) {
    return cb && ((hits[p] >> (cb - vp8l::kMinCacheBits)) & 1u);
}

__global__ __launch_bounds__(256) void k_vp8l_hist(const uint32_t *__restrict__ resid,
                                                   const uint16_t *__restrict__ tok, uint64_t npix, int w, int gw,
                                                   const uint8_t *__restrict__ gflag,
                                                   const uint8_t *__restrict__ rgba, int stride,
                                                   const uint8_t *__restrict__ hits, int cb,
                                                   uint32_t *__restrict__ hist, uint32_t *__restrict__ raw) {
    __shared__ uint32_t hs[CODE_GROUPS * vp8l::kTabSize];
    __shared__ uint32_t hr[4 * 256];
    for (int i = threadIdx.x; i < CODE_GROUPS * vp8l::kTabSize; i += 256) hs[i] = 0;
    for (int i = threadIdx.x; i < 4 * 256; i += 256) hr[i] = 0;
    __syncthreads();
    const uint64_t stride_ = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < npix; i += stride_) {
        if (raw) {
            const uint32_t y = (uint32_t)i / (uint32_t)w, x = (uint32_t)i - y * (uint32_t)w;
            const uint32_t v = sub_pixels(to_argb(*(const uint32_t *)(rgba + (size_t)y * stride + (size_t)x * 4)),
                                          0xff000000u);
            atomicAdd(&hr[0 * 256 + ((v >> 8) & 0xff)], 1u);
            atomicAdd(&hr[1 * 256 + ((v >> 16) & 0xff)], 1u);
            atomicAdd(&hr[2 * 256 + (v & 0xff)], 1u);
            atomicAdd(&hr[3 * 256 + (v >> 24)], 1u);
        }
        const uint32_t t = tok[i];
        if (t == TOK_COVERED) continue;
        uint32_t *H = hs + group_of(gflag, (uint32_t)i, w, gw) * vp8l::kTabSize;
        if (t != TOK_LIT) {
            uint32_t lp, ne, ex;
            prefix_of(t, lp, ne, ex);
            atomicAdd(&H[vp8l::kOffG + 256 + lp], 1u);
            atomicAdd(&H[vp8l::kOffD + DIST_LEFT_PREFIX], 1u);
            continue;
        }
        const uint32_t r = resid[i];
        if (cc_hit(hits, i, cb)) {
            atomicAdd(&H[vp8l::kOffG + vp8l::kGreenAlphabet + cc_index(r, cb)], 1u);
            continue;
        }
        atomicAdd(&H[vp8l::kOffG + ((r >> 8) & 0xff)], 1u);
        atomicAdd(&H[vp8l::kOffR + ((r >> 16) & 0xff)], 1u);
        atomicAdd(&H[vp8l::kOffB + (r & 0xff)], 1u);
        atomicAdd(&H[vp8l::kOffA + (r >> 24)], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < CODE_GROUPS * vp8l::kTabSize; i += 256)
        if (hs[i]) atomicAdd(&hist[i], hs[i]);
    if (raw) {
        const int off[4] = {vp8l::kOffG, vp8l::kOffR, vp8l::kOffB, vp8l::kOffA};
        for (int i = threadIdx.x; i < 4 * 256; i += 256)
            if (hr[i]) atomicAdd(&raw[off[i >> 8] + (i & 255)], hr[i]);
    }
}


// code of one token: (bits, length) LSB-first -- a literal's G, R, B, A codes, or a copy's
// length prefix (green alphabet), length extra bits and distance prefix (no extra bits)
__device__ inline uint64_t token_code(const uint32_t *tab, uint32_t r, uint32_t t, bool hit, int cb, int &n) {
    if (t == TOK_COVERED) {
        n = 0;
        return 0;
    }
    if (t == TOK_LIT && hit) {  // colour-cache index: one green symbol
        const uint32_t e = tab[vp8l::kOffG + vp8l::kGreenAlphabet + cc_index(r, cb)];
        n = (int)(e >> 16);
        return e & 0xffffu;
    }
    if (t != TOK_LIT) {
        uint32_t lp, ne, ex;
        prefix_of(t, lp, ne, ex);
        const uint32_t eg = tab[vp8l::kOffG + 256 + lp], ed = tab[vp8l::kOffD + DIST_LEFT_PREFIX];
        const int lg = eg >> 16, ld = ed >> 16;
        uint64_t v = (uint64_t)(eg & 0xffffu);
        v |= (uint64_t)ex << lg;
        v |= (uint64_t)(ed & 0xffffu) << (lg + (int)ne);
        n = lg + (int)ne + ld;
        return v;
    }
    const uint32_t eg = tab[vp8l::kOffG + ((r >> 8) & 0xff)], er = tab[vp8l::kOffR + ((r >> 16) & 0xff)];
    const uint32_t eb = tab[vp8l::kOffB + (r & 0xff)], ea = tab[vp8l::kOffA + (r >> 24)];
    const int lg = eg >> 16, lr = er >> 16, lb = eb >> 16, la = ea >> 16;
    uint64_t v = (uint64_t)(eg & 0xffffu);
    v |= (uint64_t)(er & 0xffffu) << lg;
    v |= (uint64_t)(eb & 0xffffu) << (lg + lr);
    v |= (uint64_t)(ea & 0xffffu) << (lg + lr + lb);
    n = lg + lr + lb + la;
    return v;
}

__device__ inline int token_len(const uint32_t *tab, uint32_t r, uint32_t t, bool hit, int cb) {
    if (t == TOK_COVERED) return 0;
    if (t == TOK_LIT && hit) return (int)(tab[vp8l::kOffG + vp8l::kGreenAlphabet + cc_index(r, cb)] >> 16);
    if (t != TOK_LIT) {
        uint32_t lp, ne, ex;
        prefix_of(t, lp, ne, ex);
        return (int)((tab[vp8l::kOffG + 256 + lp] >> 16) + ne + (tab[vp8l::kOffD + DIST_LEFT_PREFIX] >> 16));
    }
    return (int)((tab[vp8l::kOffG + ((r >> 8) & 0xff)] >> 16) + (tab[vp8l::kOffR + ((r >> 16) & 0xff)] >> 16) +
                 (tab[vp8l::kOffB + (r & 0xff)] >> 16) + (tab[vp8l::kOffA + (r >> 24)] >> 16));
}

// the tokens of one EMIT_PIX group: thread t owns EMIT_PP consecutive pixels; the first pixel
// after (before) each slice that is not a repeat comes from block suffix (prefix) scans
__global__ __launch_bounds__(256) void k_vp8l_runs(const uint32_t *__restrict__ resid, uint64_t npix,
                                                   uint16_t *__restrict__ tok, int w, int gw,
                                                   uint8_t *__restrict__ gflag) {
    __shared__ uint32_t nxt[256];
    __shared__ int prv[256];
    const int t = threadIdx.x;
    const uint64_t g0 = (uint64_t)blockIdx.x * EMIT_PIX;
    const uint32_t cnt = (uint32_t)min((uint64_t)EMIT_PIX, npix - g0);
    const uint32_t a = (uint32_t)t * EMIT_PP;
    bool dup[EMIT_PP];
    uint32_t first_nd = cnt;  // local indices; none: cnt
    int last_nd = -1;         // none: -1 (the run may start before this slice)
#pragma unroll
    for (int j = 0; j < EMIT_PP; ++j) {
        const uint32_t i = a + j;
        const uint64_t p = g0 + i;
        dup[j] = i < cnt && p > 0 && resid[p] == resid[p - 1];
        if (i < cnt && !dup[j]) {
            if (first_nd == cnt) first_nd = i;
            last_nd = (int)i;
        }
    }
    // nxt[t] = first non-repeat at or after slice t; prv[t] = last non-repeat at or before slice t
    nxt[t] = first_nd;
    prv[t] = last_nd;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {
        const uint32_t vn = t + o < 256 ? nxt[t + o] : cnt;
        const int vp = t >= o ? prv[t - o] : -1;
        __syncthreads();
        nxt[t] = min(nxt[t], vn);
        prv[t] = max(prv[t], vp);
        __syncthreads();
    }
    uint32_t nb = t + 1 < 256 ? nxt[t + 1] : cnt;  // first non-repeat after this slice
    int pb = t > 0 ? prv[t - 1] : -1;              // last non-repeat before this slice
    uint32_t nbr[EMIT_PP];
#pragma unroll
    for (int j = EMIT_PP - 1; j >= 0; --j) {  // first non-repeat strictly after a + j
        nbr[j] = nb;
        if (a + j < cnt && !dup[j]) nb = a + j;
    }
#pragma unroll
    for (int j = 0; j < EMIT_PP; ++j) {
        const uint32_t i = a + j;
        if (i >= cnt) break;
        uint16_t v = TOK_LIT;
        if (dup[j]) {
            const uint32_t s = (uint32_t)(pb + 1);  // the run's first repeat
            const uint32_t L = nbr[j] - s;
            if (L >= RUN_MIN) v = i == s ? (uint16_t)L : TOK_COVERED;
        } else {
            pb = (int)i;
        }
        tok[g0 + i] = v;
        if (v == TOK_LIT && (resid[g0 + i] >> 24) != 0u) {  // a literal alpha residual: group 1
            const uint32_t p = (uint32_t)(g0 + i), y = p / (uint32_t)w, x = p - y * (uint32_t)w;
            gflag[(y >> GROUP_BITS) * (uint32_t)gw + (x >> GROUP_BITS)] = 1;
        }
    }
}

__global__ __launch_bounds__(256) void k_vp8l_bits(const uint32_t *__restrict__ resid,
                                                   const uint16_t *__restrict__ tok, uint64_t npix, int w, int gw,
                                                   const uint8_t *__restrict__ gflag, int ngroups,
                                                   const uint8_t *__restrict__ hits, int cb,
                                                   const uint32_t *__restrict__ tab_g, uint32_t *__restrict__ wg_bits) {
    __shared__ uint32_t tab[CODE_GROUPS * vp8l::kTabSize];
    __shared__ uint32_t red[4];
    for (int i = threadIdx.x; i < ngroups * vp8l::kTabSize; i += 256) tab[i] = tab_g[i];
    __syncthreads();
    const uint64_t p0 = (uint64_t)blockIdx.x * EMIT_PIX + (uint64_t)threadIdx.x * EMIT_PP;
    uint32_t bits = 0;
    for (int j = 0; j < EMIT_PP; ++j)
        if (p0 + j < npix) {
            const uint32_t g = ngroups > 1 ? group_of(gflag, (uint32_t)(p0 + j), w, gw) : 0u;
            bits += token_len(tab + g * vp8l::kTabSize, resid[p0 + j], tok[p0 + j], cc_hit(hits, p0 + j, cb), cb);
        }
    for (int o = 32; o > 0; o >>= 1) bits += __shfl_xor(bits, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = bits;
    __syncthreads();
    if (threadIdx.x == 0) wg_bits[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// exclusive bit offsets of the groups, starting at `start`; also the RIFF/VP8L sizes
// (bytes 4..7 and 16..19 of the file) and the file size
__global__ __launch_bounds__(1024) void k_vp8l_scan(const uint32_t *__restrict__ wg_bits, uint32_t nwg, uint64_t start,
                                                    uint64_t *__restrict__ wg_off, uint8_t *__restrict__ file,
                                                    uint64_t *__restrict__ file_size) {
    __shared__ uint64_t part[1024];
    const uint32_t per = (nwg + 1023) / 1024;
    const uint32_t b0 = threadIdx.x * per, b1 = min(nwg, b0 + per);
    uint64_t s = 0;
    for (uint32_t i = b0; i < b1; ++i) s += wg_bits[i];
    part[threadIdx.x] = s;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const uint64_t v = threadIdx.x >= (unsigned)o ? part[threadIdx.x - o] : 0;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    uint64_t run = start + part[threadIdx.x] - s;
    for (uint32_t i = b0; i < b1; ++i) {
        wg_off[i] = run;
        run += wg_bits[i];
    }
    if (threadIdx.x == 1023) {
        const uint64_t end_bits = start + part[1023];                // bits from the file start
        const uint64_t vp8l_bytes = (end_bits - 20 * 8 + 7) / 8;     // VP8L chunk payload
        const uint64_t pad = vp8l_bytes & 1;
        const uint64_t riff = 4 + 8 + vp8l_bytes + pad;
        for (int k = 0; k < 4; ++k) {
            file[4 + k] = (uint8_t)(riff >> (8 * k));
            file[16 + k] = (uint8_t)(vp8l_bytes >> (8 * k));
        }
        wg_off[nwg] = end_bits;
        *file_size = 8 + riff;
    }
}

__global__ __launch_bounds__(256) void k_vp8l_emit(const uint32_t *__restrict__ resid,
                                                   const uint16_t *__restrict__ tok, uint64_t npix, int w, int gw,
                                                   const uint8_t *__restrict__ gflag, int ngroups,
                                                   const uint8_t *__restrict__ hits, int cb,
                                                   const uint32_t *__restrict__ tab_g,
                                                   const uint64_t *__restrict__ wg_off, uint32_t *__restrict__ out) {
    __shared__ uint32_t tab[CODE_GROUPS * vp8l::kTabSize];
    __shared__ uint32_t words[EMIT_WORDS];
    __shared__ uint32_t tsum[256];
    for (int i = threadIdx.x; i < ngroups * vp8l::kTabSize; i += 256) tab[i] = tab_g[i];
    for (int i = threadIdx.x; i < EMIT_WORDS; i += 256) words[i] = 0;
    __syncthreads();
    const uint64_t p0 = (uint64_t)blockIdx.x * EMIT_PIX + (uint64_t)threadIdx.x * EMIT_PP;
    uint32_t r[EMIT_PP], tk[EMIT_PP], gt[EMIT_PP];
    bool hb[EMIT_PP];
    uint32_t mine = 0;
#pragma unroll
    for (int j = 0; j < EMIT_PP; ++j) {
        r[j] = (p0 + j < npix) ? resid[p0 + j] : 0u;
        tk[j] = (p0 + j < npix) ? tok[p0 + j] : TOK_COVERED;
        gt[j] = (ngroups > 1 && p0 + j < npix) ? group_of(gflag, (uint32_t)(p0 + j), w, gw) * vp8l::kTabSize : 0u;
        hb[j] = p0 + j < npix && cc_hit(hits, p0 + j, cb);
        if (p0 + j < npix) mine += token_len(tab + gt[j], r[j], tk[j], hb[j], cb);
    }
    // inclusive scan of the threads' bit counts
    tsum[threadIdx.x] = mine;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {
        const uint32_t v = threadIdx.x >= (unsigned)o ? tsum[threadIdx.x - o] : 0;
        __syncthreads();
        tsum[threadIdx.x] += v;
        __syncthreads();
    }
    const uint64_t base = wg_off[blockIdx.x];
    const uint32_t total = tsum[255];
    const uint32_t sh = (uint32_t)(base & 31);
    uint32_t pos = sh + tsum[threadIdx.x] - mine;
#pragma unroll
    for (int j = 0; j < EMIT_PP; ++j) {
        if (p0 + j >= npix) break;
        int n;
        const uint64_t v = token_code(tab + gt[j], r[j], tk[j], hb[j], cb, n);
        if (n) {
            const uint32_t wi = pos >> 5, s = pos & 31;
            atomicOr(&words[wi], (uint32_t)(v << s));
            const uint64_t rest = s ? (v >> (32 - s)) : (v >> 32);
            if (s + n > 32) atomicOr(&words[wi + 1], (uint32_t)rest);
            if (s + n > 64) atomicOr(&words[wi + 2], (uint32_t)(rest >> 32));
            pos += n;
        }
    }
    __syncthreads();
    const uint32_t nwords = (sh + total + 31) >> 5;
    uint32_t *dst = out + (base >> 5);
    for (uint32_t j = threadIdx.x; j < nwords; j += 256) {
        if (j == 0 || j == nwords - 1)
            atomicOr(&dst[j], words[j]);  // shared with the neighbouring run (or the header)
        else
            dst[j] = words[j];
    }
}

// ---- colour cache ----------------------------------------------------------------
constexpr int CC_SLOTS = vp8l::kCacheSlots;  // the slots of every candidate size, cache_off layout
constexpr uint32_t CC_CHUNK = 64;            // groups per carry-scan chunk
constexpr uint64_t CC_SET = 1ull << 32;      // a table entry: CC_SET | colour once written, else 0

// W[g][j]: the colour of the last pixel of group g with cache slot j (every candidate size at
// once), CC_SET | colour, or 0 when no pixel of the group has that slot: the largest position per
// slot by LDS atomicMax, then its colour
__global__ __launch_bounds__(256) void k_cc_tab(const uint32_t *__restrict__ resid, uint64_t npix,
                                                uint64_t *__restrict__ W) {
    __shared__ uint32_t last[CC_SLOTS];
    for (int j = threadIdx.x; j < CC_SLOTS; j += 256) last[j] = 0;
    __syncthreads();
    const uint64_t g0 = (uint64_t)blockIdx.x * EMIT_PIX;
    const uint32_t cnt = (uint32_t)min((uint64_t)EMIT_PIX, npix - g0);
    for (uint32_t i = threadIdx.x; i < cnt; i += 256) {
        const uint32_t h = resid[g0 + i] * vp8l::kCacheMul;
#pragma unroll
        for (int l = 0; l < vp8l::kCacheLevels; ++l) {
            const int bits = vp8l::kMinCacheBits + l;
            atomicMax(&last[vp8l::cache_off(bits) + (h >> (32 - bits))], i + 1);
        }
    }
    __syncthreads();
    uint64_t *Wg = W + (uint64_t)blockIdx.x * CC_SLOTS;
    for (int j = threadIdx.x; j < CC_SLOTS; j += 256) {
        const uint32_t q = last[j];
        Wg[j] = q ? (CC_SET | resid[g0 + q - 1]) : 0ull;
    }
}

// W[g][j] <- the last written entry of the groups before g in g's chunk (0: none); A[chunk][j] <-
// the chunk's last written entry
__global__ __launch_bounds__(256) void k_cc_scan1(uint64_t *__restrict__ W, uint32_t ngroups,
                                                  uint64_t *__restrict__ A) {
    const uint32_t j = blockIdx.x * 256 + threadIdx.x;
    if (j >= (uint32_t)CC_SLOTS) return;
    const uint32_t g0 = blockIdx.y * CC_CHUNK, g1 = min(ngroups, g0 + CC_CHUNK);
    uint64_t carry = 0;
    for (uint32_t g = g0; g < g1; ++g) {
        const uint64_t v = W[(uint64_t)g * CC_SLOTS + j];
        W[(uint64_t)g * CC_SLOTS + j] = carry;
        if (v) carry = v;
    }
    A[(uint64_t)blockIdx.y * CC_SLOTS + j] = carry;
}

// A[chunk][j] <- the last written entry of the chunks before it (0: none)
__global__ __launch_bounds__(256) void k_cc_scan2(uint64_t *__restrict__ A, uint32_t nchunks) {
    const uint32_t j = blockIdx.x * 256 + threadIdx.x;
    if (j >= (uint32_t)CC_SLOTS) return;
    uint64_t carry = 0;
    for (uint32_t q = 0; q < nchunks; ++q) {
        const uint64_t v = A[(uint64_t)q * CC_SLOTS + j];
        A[(uint64_t)q * CC_SLOTS + j] = carry;
        if (v) carry = v;
    }
}

// one wave per EMIT_PIX group; lane l < kCacheLevels replays the 2^(kMinCacheBits + l)-entry cache
// over the group's pixels in order, starting from the cache as the earlier groups left it (the
// scans).  A slot no earlier pixel wrote starts with a colour whose own index is another slot, so
// no pixel can match it (the zero-initialised cache is not relied on): hits[p] bit l exactly when
// the last earlier pixel with p's index has p's colour.
__global__ __launch_bounds__(64) void k_cc_walk(const uint32_t *__restrict__ resid, uint64_t npix,
                                                const uint64_t *__restrict__ W, const uint64_t *__restrict__ A,
                                                uint8_t *__restrict__ hits) {
    // lanes >= kCacheLevels replay nothing: they read and write a private slot past the table,
    // so the step loop has no exec-mask branches
    __shared__ uint32_t cache[CC_SLOTS + 64];
    const int lane = threadIdx.x;
    const uint64_t g = blockIdx.x;
    for (int j = lane; j < CC_SLOTS; j += 64) {
        uint64_t e = W[g * CC_SLOTS + j];
        if (!e) e = A[(g / CC_CHUNK) * CC_SLOTS + j];
        const int bits = 31 - __builtin_clz((uint32_t)j + (1u << vp8l::kMinCacheBits));
        const uint32_t idx = (uint32_t)j - (uint32_t)vp8l::cache_off(bits);
        // index(0) = 0 and index(1) = 0x1e35a7bd >> (32 - bits) != 0: 1 where index 0, else 0
        cache[j] = e ? (uint32_t)e : (idx == 0 ? 1u : 0u);
    }
    cache[CC_SLOTS + lane] = 0;
    __syncthreads();
    const uint64_t g0 = g * EMIT_PIX;
    const uint32_t cnt = (uint32_t)min((uint64_t)EMIT_PIX, npix - g0);
    const bool act = lane < vp8l::kCacheLevels;
    const int bits = vp8l::kMinCacheBits + (act ? lane : 0);
    const uint32_t base = (uint32_t)vp8l::cache_off(bits), own = (uint32_t)CC_SLOTS + lane;
    constexpr uint32_t LEVEL_MASK = (1u << vp8l::kCacheLevels) - 1;
    constexpr int SUB = 16;  // steps whose LDS reads and writes are issued before their compares
    for (uint32_t i0 = 0; i0 < cnt; i0 += 64) {
        const uint32_t m = min(64u, cnt - i0);
        const uint32_t pv = (uint32_t)lane < m ? resid[g0 + i0 + lane] : 0u;
        uint32_t mine = 0;  // lane q: the hit bits of pixel i0 + q
        if (m == 64) {
#pragma unroll
            for (int k0 = 0; k0 < 64; k0 += SUB) {
                uint32_t e[SUB];
#pragma unroll
                for (int u = 0; u < SUB; ++u) {
                    const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)pv, k0 + u);
                    const uint32_t slot = act ? base + cc_index(c, bits) : own;
                    e[u] = cache[slot];
                    cache[slot] = c;
                }
#pragma unroll
                for (int u = 0; u < SUB; ++u) {
                    const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)pv, k0 + u);
                    const uint32_t hm = (uint32_t)__ballot(e[u] == c) & LEVEL_MASK;
                    mine = lane == k0 + u ? hm : mine;
                }
            }
        } else {  // the image's last, partial batch: one step at a time
            for (uint32_t k = 0; k < m; ++k) {
                const uint32_t c = (uint32_t)__shfl((int)pv, (int)k, 64);
                const uint32_t slot = act ? base + cc_index(c, bits) : own;
                const uint32_t e = cache[slot];
                cache[slot] = c;
                const uint32_t hm = (uint32_t)__ballot(e == c) & LEVEL_MASK;
                mine = (uint32_t)lane == k ? hm : mine;
            }
        }
        if ((uint32_t)lane < m) hits[g0 + i0 + lane] = (uint8_t)mine;
    }
}

// per cache size, the literals that hit it: hitlit[l] = the G, R, B, A values of the literals
// whose smallest hitting size is level l; cidx = their indices at every level they hit
__global__ __launch_bounds__(256) void k_cc_survey(const uint32_t *__restrict__ resid,
                                                   const uint16_t *__restrict__ tok, const uint8_t *__restrict__ hits,
                                                   uint64_t npix, uint32_t *__restrict__ hitlit,
                                                   uint32_t *__restrict__ cidx) {
    __shared__ uint32_t hl[vp8l::kCacheLevels * 1024];
    __shared__ uint32_t ci[CC_SLOTS];
    for (int i = threadIdx.x; i < vp8l::kCacheLevels * 1024; i += 256) hl[i] = 0;
    for (int i = threadIdx.x; i < CC_SLOTS; i += 256) ci[i] = 0;
    __syncthreads();
    const uint64_t stride_ = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < npix; i += stride_) {
        const uint32_t m = hits[i];
        if (!m || tok[i] != TOK_LIT) continue;
        const uint32_t r = resid[i];
        const int l0 = __builtin_ctz(m);
        uint32_t *h = hl + l0 * 1024;
        atomicAdd(&h[(r >> 8) & 0xff], 1u);
        atomicAdd(&h[256 + ((r >> 16) & 0xff)], 1u);
        atomicAdd(&h[512 + (r & 0xff)], 1u);
        atomicAdd(&h[768 + (r >> 24)], 1u);
        for (int l = l0; l < vp8l::kCacheLevels; ++l) {
            const int bits = vp8l::kMinCacheBits + l;
            atomicAdd(&ci[vp8l::cache_off(bits) + cc_index(r, bits)], 1u);
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < vp8l::kCacheLevels * 1024; i += 256)
        if (hl[i]) atomicAdd(&hitlit[i], hl[i]);
    for (int i = threadIdx.x; i < CC_SLOTS; i += 256)
        if (ci[i]) atomicAdd(&cidx[i], ci[i]);
}

// ---- CRC-32 (zlib polynomial, reflected) ---------------------------------------
constexpr uint32_t CRC_POLY = 0xedb88320u;
constexpr uint32_t CRC_SPAN = 2048;  // bytes per thread

__host__ __device__ inline uint32_t multmodp(uint32_t a, uint32_t b) {
    uint32_t m = 1u << 31, p = 0;
    for (;;) {
        if (a & m) {
            p ^= b;
            if ((a & (m - 1)) == 0) break;
        }
        m >>= 1;
        b = (b & 1) ? (b >> 1) ^ CRC_POLY : b >> 1;
    }
    return p;
}

// x^(n * 2^k) mod P, with x2n[i] = x^(2^i)
__host__ __device__ inline uint32_t x2nmodp(const uint32_t *x2n, uint64_t n, unsigned k) {
    uint32_t p = 1u << 31;  // x^0
    while (n) {
        if (n & 1) p = multmodp(x2n[k & 31], p);
        n >>= 1;
        ++k;
    }
    return p;
}

__global__ __launch_bounds__(256) void k_crc32(const uint8_t *__restrict__ data, uint64_t n, uint32_t init,
                                               uint32_t *__restrict__ out) {
    // slicing-by-8: tbl[k][b] = CRC of byte b followed by k zero bytes
    __shared__ uint32_t tbl[8][256];
    __shared__ uint32_t x2n[32];
    __shared__ uint32_t red[4];
    {
        uint32_t c = threadIdx.x;
        for (int k = 0; k < 8; ++k) c = (c & 1) ? (CRC_POLY ^ (c >> 1)) : (c >> 1);
        tbl[0][threadIdx.x] = c;
    }
    if (threadIdx.x == 0) {
        uint32_t p = 1u << 30;  // x^1
        x2n[0] = p;
        for (int i = 1; i < 32; ++i) x2n[i] = p = multmodp(p, p);
    }
    __syncthreads();
    for (int k = 1; k < 8; ++k) {
        const uint32_t v = tbl[k - 1][threadIdx.x];
        tbl[k][threadIdx.x] = (v >> 8) ^ tbl[0][v & 0xff];
        __syncthreads();
    }
    const uint64_t s0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * CRC_SPAN;
    uint32_t contrib = 0;
    if (s0 < n) {
        const uint64_t s1 = (s0 + CRC_SPAN < n) ? s0 + CRC_SPAN : n;
        uint32_t c = 0xffffffffu;
        uint64_t i = s0;
        for (; i < s1 && (((uintptr_t)data + i) & 15); ++i) c = (c >> 8) ^ tbl[0][(c ^ data[i]) & 0xff];
        auto step8 = [&](uint32_t lo, uint32_t hi) {
            c ^= lo;
            c = tbl[7][c & 0xff] ^ tbl[6][(c >> 8) & 0xff] ^ tbl[5][(c >> 16) & 0xff] ^ tbl[4][c >> 24] ^
                tbl[3][hi & 0xff] ^ tbl[2][(hi >> 8) & 0xff] ^ tbl[1][(hi >> 16) & 0xff] ^ tbl[0][hi >> 24];
        };
        for (; i + 16 <= s1; i += 16) {
            const uint4 q = *(const uint4 *)(data + i);
            step8(q.x, q.y);
            step8(q.z, q.w);
        }
        for (; i < s1; ++i) c = (c >> 8) ^ tbl[0][(c ^ data[i]) & 0xff];
        c ^= 0xffffffffu;
        // crc(A B) = crc(A) * x^(8|B|) xor crc(B): shift this span's CRC to the end of the buffer
        contrib = multmodp(x2nmodp(x2n, n - s1, 3), c);
    }
    for (int o = 32; o > 0; o >>= 1) contrib ^= __shfl_xor(contrib, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = contrib;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t v = red[0] ^ red[1] ^ red[2] ^ red[3];
        if (blockIdx.x == 0) v ^= init;
        atomicXor(out, v);
    }
}

uint32_t host_x2n[32];
bool host_x2n_ready = false;

void init_host_x2n() {
    if (host_x2n_ready) return;
    uint32_t p = 1u << 30;
    host_x2n[0] = p;
    for (int i = 1; i < 32; ++i) host_x2n[i] = p = multmodp(p, p);
    host_x2n_ready = true;
}

}  // namespace

uint64_t webp_max_size(int w, int h) {
    // header: RIFF 20 B + <= 4 KiB of code descriptions + the predictor sub-image
    // (<= 15 bits per block); pixels <= 60 bits; + word slack for the emitter
    const uint64_t npix = (uint64_t)w * h;
    const uint64_t blocks = (uint64_t)((w + PB - 1) / PB) * ((h + PB - 1) / PB);
    return 20 + 4096 + (blocks * 15 + 7) / 8 + (npix * 60 + 7) / 8 + 16;
}

// host work of several images at once (prefix codes, headers): one thread per image, the
// first exception rethrown after all have joined
template <typename F>
static void per_job(int njobs, F fn) {
    std::vector<std::thread> th;
    std::vector<std::exception_ptr> err(njobs);
    for (int j = 0; j < njobs; ++j)
        th.emplace_back([&, j] {
            try {
                fn(j);
            } catch (...) {
                err[j] = std::current_exception();
            }
        });
    for (auto &t : th) t.join();
    for (auto &e : err)
        if (e) std::rethrow_exception(e);
}

void webp_encode_dev(st_ctx *c, WebpJob *jobs, int njobs) {
    // per job in pinned staging: group histograms, the raw histogram, predictor modes, group
    // flags, the colour-cache survey (hit literals per size, cache indices)
    struct Stage {
        size_t hist, raw, modes, flags, hitlit, cidx;
    };
    std::vector<Stage> stage;
    size_t pin = 0;
    auto geom = [](const WebpJob &jb, int &bw, int &bh, int &gw, int &gh) {
        bw = (jb.w + PB - 1) / PB, bh = (jb.h + PB - 1) / PB;
        gw = (jb.w + (1 << GROUP_BITS) - 1) >> GROUP_BITS, gh = (jb.h + (1 << GROUP_BITS) - 1) >> GROUP_BITS;
    };
    for (int j = 0; j < njobs; ++j) {
        WebpJob &jb = jobs[j];
        ST_REQUIRE(jb.w >= 1 && jb.h >= 1 && jb.w <= 16384 && jb.h <= 16384, ST_ERR_ARG,
                   "webp: image size must be 1..16384");
        ST_REQUIRE(jb.stride >= jb.w * 4 && jb.stride % 4 == 0 && ((uintptr_t)jb.rgba & 3) == 0, ST_ERR_ARG,
                   "webp: rgba rows must be 4-byte aligned");
        ST_REQUIRE(((uintptr_t)jb.out & 3) == 0, ST_ERR_ARG, "webp: output must be 4-byte aligned");
        ST_REQUIRE(jb.cap >= webp_max_size(jb.w, jb.h), ST_ERR_ARG, "webp: output capacity below st_webp_max_size");
        int bw, bh, gw, gh;
        geom(jb, bw, bh, gw, gh);
        Stage st;
        st.hist = pin;
        st.raw = st.hist + CODE_GROUPS * vp8l::kTabSize * 4;
        st.modes = st.raw + vp8l::kTabSize * 4;
        st.flags = st.modes + (size_t)bw * bh;
        st.hitlit = (st.flags + (size_t)gw * gh + 15) & ~(size_t)15;
        st.cidx = st.hitlit + (size_t)vp8l::kCacheLevels * 1024 * 4;
        stage.push_back(st);
        pin = (st.cidx + (size_t)CC_SLOTS * 4 + 255) & ~(size_t)255;
    }
    // colour-cache tables, shared by the jobs (one stream: each job's tables, scans and walk run
    // before the next job's)
    uint32_t max_groups = 1;
    for (int j = 0; j < njobs; ++j)
        max_groups = std::max(max_groups, (uint32_t)(((uint64_t)jobs[j].w * jobs[j].h + EMIT_PIX - 1) / EMIT_PIX));
    uint64_t *ccW = wsT<uint64_t>(c, "wp.ccw", (size_t)max_groups * CC_SLOTS);
    uint64_t *ccA = wsT<uint64_t>(c, "wp.cca", (size_t)((max_groups + CC_CHUNK - 1) / CC_CHUNK) * CC_SLOTS);
    // phase A: predictors, residuals, tokens, group flags, histograms (raw = the pixels as no
    // predictor leaves them, for the choice below)
    auto phase_a = [&](int j, int force_mode) {
        WebpJob &jb = jobs[j];
        const std::string tag = "wp" + std::to_string(j);
        int bw, bh, gw, gh;
        geom(jb, bw, bh, gw, gh);
        const uint64_t npix = (uint64_t)jb.w * jb.h;
        uint32_t *resid = wsT<uint32_t>(c, tag + ".res", npix);
        uint8_t *modes = wsT<uint8_t>(c, tag + ".modes", (size_t)bw * bh);
        uint32_t *hist = wsT<uint32_t>(c, tag + ".hist", (size_t)CODE_GROUPS * vp8l::kTabSize);
        uint32_t *raw = wsT<uint32_t>(c, tag + ".raw", vp8l::kTabSize);
        uint16_t *tok = wsT<uint16_t>(c, tag + ".tok", npix);
        uint8_t *gflag = wsT<uint8_t>(c, tag + ".gfl", (size_t)gw * gh);
        ST_HIP(hipMemsetAsync(hist, 0, (size_t)CODE_GROUPS * vp8l::kTabSize * 4, c->stream));
        ST_HIP(hipMemsetAsync(raw, 0, vp8l::kTabSize * 4, c->stream));
        ST_HIP(hipMemsetAsync(gflag, 0, (size_t)gw * gh, c->stream));
        {
            KTimer kt(c, "webp.predict");
            hipLaunchKernelGGL(k_vp8l_predict, dim3(bw * bh), dim3(256), 0, c->stream, jb.rgba, jb.w, jb.h, jb.stride,
                               bw, modes, resid, force_mode);
            ST_LAUNCH_CHECK();
        }
        {
            KTimer kt(c, "webp.hist");
            hipLaunchKernelGGL(k_vp8l_runs, dim3((unsigned)((npix + EMIT_PIX - 1) / EMIT_PIX)), dim3(256), 0,
                               c->stream, resid, npix, tok, jb.w, gw, gflag);
            hipLaunchKernelGGL(k_vp8l_hist, dim3(grid_for(npix, 256 * 16, 2048)), dim3(256), 0, c->stream, resid, tok,
                               npix, jb.w, gw, gflag, jb.rgba, jb.stride, (const uint8_t *)nullptr, 0, hist,
                               force_mode < 0 ? raw : nullptr);
            ST_LAUNCH_CHECK();
        }
        uint8_t *hp = (uint8_t *)pinned(c, pin);
        ST_HIP(hipMemcpyAsync(hp + stage[j].hist, hist, (size_t)CODE_GROUPS * vp8l::kTabSize * 4,
                              hipMemcpyDeviceToHost, c->stream));
        ST_HIP(hipMemcpyAsync(hp + stage[j].raw, raw, vp8l::kTabSize * 4, hipMemcpyDeviceToHost, c->stream));
        ST_HIP(hipMemcpyAsync(hp + stage[j].modes, modes, (size_t)bw * bh, hipMemcpyDeviceToHost, c->stream));
        ST_HIP(hipMemcpyAsync(hp + stage[j].flags, gflag, (size_t)gw * gh, hipMemcpyDeviceToHost, c->stream));
    };
    // the colour cache of the final residuals: hits for every candidate size, the survey
    auto cache_stage = [&](int j) {
        WebpJob &jb = jobs[j];
        const std::string tag = "wp" + std::to_string(j);
        const uint64_t npix = (uint64_t)jb.w * jb.h;
        const uint32_t ngrp = (uint32_t)((npix + EMIT_PIX - 1) / EMIT_PIX);
        const uint32_t *resid = wsT<uint32_t>(c, tag + ".res", npix);
        const uint16_t *tok = wsT<uint16_t>(c, tag + ".tok", npix);
        uint8_t *hits = wsT<uint8_t>(c, tag + ".cch", (size_t)ngrp * EMIT_PIX);
        uint32_t *hitlit = wsT<uint32_t>(c, tag + ".chl", (size_t)vp8l::kCacheLevels * 1024);
        uint32_t *cidx = wsT<uint32_t>(c, tag + ".cci", (size_t)CC_SLOTS);
        ST_HIP(hipMemsetAsync(hitlit, 0, (size_t)vp8l::kCacheLevels * 1024 * 4, c->stream));
        ST_HIP(hipMemsetAsync(cidx, 0, (size_t)CC_SLOTS * 4, c->stream));
        {
            KTimer kt(c, "webp.cache");
            const uint32_t nch = (ngrp + CC_CHUNK - 1) / CC_CHUNK;
            const unsigned sb = (CC_SLOTS + 255) / 256;
            hipLaunchKernelGGL(k_cc_tab, dim3(ngrp), dim3(256), 0, c->stream, resid, npix, ccW);
            hipLaunchKernelGGL(k_cc_scan1, dim3(sb, nch), dim3(256), 0, c->stream, ccW, ngrp, ccA);
            hipLaunchKernelGGL(k_cc_scan2, dim3(sb), dim3(256), 0, c->stream, ccA, nch);
            hipLaunchKernelGGL(k_cc_walk, dim3(ngrp), dim3(64), 0, c->stream, resid, npix, ccW, ccA, hits);
            hipLaunchKernelGGL(k_cc_survey, dim3(grid_for(npix, 256 * 16, 2048)), dim3(256), 0, c->stream, resid, tok,
                               hits, npix, hitlit, cidx);
            ST_LAUNCH_CHECK();
        }
        uint8_t *hp = (uint8_t *)pinned(c, pin);
        ST_HIP(hipMemcpyAsync(hp + stage[j].hitlit, hitlit, (size_t)vp8l::kCacheLevels * 1024 * 4,
                              hipMemcpyDeviceToHost, c->stream));
        ST_HIP(hipMemcpyAsync(hp + stage[j].cidx, cidx, (size_t)CC_SLOTS * 4, hipMemcpyDeviceToHost, c->stream));
    };
    for (int j = 0; j < njobs; ++j) phase_a(j, -1);
    ST_HIP(hipStreamSynchronize(c->stream));
    // per image: when the pixels themselves code in fewer literal bits than the chosen
    // predictors' residuals (no spatial correlation: codebook indices of independent
    // attributes), predict nothing (mode 0 everywhere) and redo phase A for that image
    uint8_t *hp = (uint8_t *)pinned(c, pin);
    bool again = false;
    std::vector<int> forced(njobs, 0);
    for (int j = 0; j < njobs; ++j) {
        const uint32_t *h = (const uint32_t *)(hp + stage[j].hist);
        const double sel = vp8l::literal_bits(h) + vp8l::literal_bits(h + vp8l::kTabSize);
        const double raw = vp8l::literal_bits((const uint32_t *)(hp + stage[j].raw));
        if (raw < 0.995 * sel) {
            forced[j] = 1;
            again = true;
        }
    }
    if (again)
        for (int j = 0; j < njobs; ++j)
            if (forced[j]) phase_a(j, 0);
    bool any_cache = false;
    for (int j = 0; j < njobs; ++j)
        if (jobs[j].cache) {
            cache_stage(j);
            any_cache = true;
        }
    if (any_cache) ST_HIP(hipStreamSynchronize(c->stream));
    // per image: the colour-cache size; with a cache, the histograms again (a hitting literal is
    // one green symbol)
    std::vector<int> cbits(njobs, 0);
    per_job(njobs, [&](int j) {
        const uint32_t *h = (const uint32_t *)(hp + stage[j].hist);
        std::vector<uint32_t> merged(vp8l::kTabSize);
        for (int q = 0; q < vp8l::kTabSize; ++q) merged[q] = h[q] + h[vp8l::kTabSize + q];
        if (jobs[j].cache)
            cbits[j] = vp8l::choose_cache_bits(merged.data(), (const uint32_t *)(hp + stage[j].hitlit),
                                               (const uint32_t *)(hp + stage[j].cidx));
    });
    bool rehist = false;
    for (int j = 0; j < njobs; ++j) {
        if (getenv("ST_DEBUG"))
            fprintf(stderr, "[st webp] image %d (%d x %d): predictor %s, colour cache bits %d\n", j, jobs[j].w,
                    jobs[j].h, forced[j] ? "none" : "per block", cbits[j]);
        if (!cbits[j]) continue;
        rehist = true;
        WebpJob &jb = jobs[j];
        const std::string tag = "wp" + std::to_string(j);
        int bw, bh, gw, gh;
        geom(jb, bw, bh, gw, gh);
        const uint64_t npix = (uint64_t)jb.w * jb.h;
        const uint32_t ngrp = (uint32_t)((npix + EMIT_PIX - 1) / EMIT_PIX);
        uint32_t *hist = wsT<uint32_t>(c, tag + ".hist", (size_t)CODE_GROUPS * vp8l::kTabSize);
        ST_HIP(hipMemsetAsync(hist, 0, (size_t)CODE_GROUPS * vp8l::kTabSize * 4, c->stream));
        KTimer kt(c, "webp.hist");
        hipLaunchKernelGGL(k_vp8l_hist, dim3(grid_for(npix, 256 * 16, 2048)), dim3(256), 0, c->stream,
                           wsT<uint32_t>(c, tag + ".res", npix), wsT<uint16_t>(c, tag + ".tok", npix), npix, jb.w, gw,
                           wsT<uint8_t>(c, tag + ".gfl", (size_t)gw * gh), jb.rgba, jb.stride,
                           wsT<uint8_t>(c, tag + ".cch", (size_t)ngrp * EMIT_PIX), cbits[j], hist,
                           (uint32_t *)nullptr);
        ST_LAUNCH_CHECK();
        ST_HIP(hipMemcpyAsync(hp + stage[j].hist, hist, (size_t)CODE_GROUPS * vp8l::kTabSize * 4,
                              hipMemcpyDeviceToHost, c->stream));
    }
    if (rehist) ST_HIP(hipStreamSynchronize(c->stream));
    // host: prefix codes + header bits (two groups when some block holds a literal alpha residual)
    std::vector<vp8l::Header> hdr(njobs);
    std::vector<int> ngroups(njobs, 1);
    per_job(njobs, [&](int j) {
        int bw, bh, gw, gh;
        geom(jobs[j], bw, bh, gw, gh);
        const uint32_t *hist = (const uint32_t *)(hp + stage[j].hist);
        uint8_t *modes = hp + stage[j].modes;
        const uint8_t *flags = hp + stage[j].flags;
        bool alpha_used = false;
        for (int i = 0; i < bw * bh; ++i) {
            alpha_used = alpha_used || (modes[i] & 0x80);
            modes[i] &= 0x7f;
        }
        for (int i = 0; i < gw * gh && ngroups[j] == 1; ++i)
            if (flags[i]) ngroups[j] = CODE_GROUPS;
        if (ngroups[j] > 1) {
            vp8l::build_header(jobs[j].w, jobs[j].h, alpha_used, hist, ngroups[j], flags, GROUP_BITS, modes, cbits[j],
                               hdr[j]);
        } else {  // one group: group 1's symbols (if any) join group 0
            ngroups[j] = 1;
            std::vector<uint32_t> merged(vp8l::kTabSize);
            for (int s = 0; s < vp8l::kTabSize; ++s) merged[s] = hist[s] + hist[vp8l::kTabSize + s];
            vp8l::build_header(jobs[j].w, jobs[j].h, alpha_used, merged.data(), 1, flags, GROUP_BITS, modes, cbits[j],
                               hdr[j]);
        }
    });
    // phase C: bit counts, offsets, emission
    std::vector<std::vector<uint8_t>> head(njobs);
    std::vector<std::string> tags(njobs);
    for (int j = 0; j < njobs; ++j) {
        WebpJob &jb = jobs[j];
        tags[j] = "wp" + std::to_string(j);
        int bw, bh, gw, gh;
        geom(jb, bw, bh, gw, gh);
        const uint64_t npix = (uint64_t)jb.w * jb.h;
        const uint32_t nwg = (uint32_t)((npix + EMIT_PIX - 1) / EMIT_PIX);
        // RIFF header (sizes patched by k_vp8l_scan) + the VP8L header bits
        head[j].assign(20, 0);
        std::memcpy(head[j].data(), "RIFF", 4);
        std::memcpy(head[j].data() + 8, "WEBPVP8L", 8);
        const std::vector<uint8_t> hb = hdr[j].bw.bytes();
        head[j].insert(head[j].end(), hb.begin(), hb.end());
        uint32_t *tab = wsT<uint32_t>(c, tags[j] + ".tab", (size_t)CODE_GROUPS * vp8l::kTabSize);
        uint32_t *wg_bits = wsT<uint32_t>(c, tags[j] + ".wgb", nwg);
        uint64_t *wg_off = wsT<uint64_t>(c, tags[j] + ".wgo", (size_t)nwg + 1);
        uint64_t *fsize = wsT<uint64_t>(c, tags[j] + ".fsz", 1);
        const uint32_t *resid = wsT<uint32_t>(c, tags[j] + ".res", npix);
        const uint16_t *tok = wsT<uint16_t>(c, tags[j] + ".tok", npix);
        const uint8_t *gflag = wsT<uint8_t>(c, tags[j] + ".gfl", (size_t)gw * gh);
        const uint8_t *hits = wsT<uint8_t>(c, tags[j] + ".cch", (size_t)nwg * EMIT_PIX);
        ST_HIP(hipMemsetAsync(jb.out, 0, webp_max_size(jb.w, jb.h), c->stream));
        ST_HIP(hipMemcpyAsync(jb.out, head[j].data(), head[j].size(), hipMemcpyHostToDevice, c->stream));
        ST_HIP(hipMemcpyAsync(tab, hdr[j].tab.data(), hdr[j].tab.size() * 4, hipMemcpyHostToDevice, c->stream));
        {
            KTimer kt(c, "webp.bits");
            hipLaunchKernelGGL(k_vp8l_bits, dim3(nwg), dim3(256), 0, c->stream, resid, tok, npix, jb.w, gw, gflag,
                               ngroups[j], hits, cbits[j], tab, wg_bits);
            ST_LAUNCH_CHECK();
        }
        hipLaunchKernelGGL(k_vp8l_scan, dim3(1), dim3(1024), 0, c->stream, wg_bits, nwg,
                           (uint64_t)20 * 8 + hdr[j].bw.nbits, wg_off, jb.out, fsize);
        ST_LAUNCH_CHECK();
        {
            KTimer kt(c, "webp.emit");
            hipLaunchKernelGGL(k_vp8l_emit, dim3(nwg), dim3(256), 0, c->stream, resid, tok, npix, jb.w, gw, gflag,
                               ngroups[j], hits, cbits[j], tab, wg_off, (uint32_t *)jb.out);
            ST_LAUNCH_CHECK();
        }
    }
    uint64_t *sizes = (uint64_t *)pinned_slot(c, "wp.sizes", 8 * (size_t)njobs);
    for (int j = 0; j < njobs; ++j)
        ST_HIP(hipMemcpyAsync(sizes + j, wsT<uint64_t>(c, tags[j] + ".fsz", 1), 8, hipMemcpyDeviceToHost, c->stream));
    ST_HIP(hipStreamSynchronize(c->stream));  // also keeps head[] alive until the copies ran
    for (int j = 0; j < njobs; ++j) jobs[j].size = sizes[j];
}

void crc32_dev(st_ctx *c, const uint8_t *const *data, const uint64_t *n, const uint32_t *crc_in, int cnt,
               uint32_t *crcs) {
    init_host_x2n();
    uint32_t *d = wsT<uint32_t>(c, "crc.out", (size_t)cnt);
    ST_HIP(hipMemsetAsync(d, 0, 4 * (size_t)cnt, c->stream));
    for (int j = 0; j < cnt; ++j) {
        // crc32(c0, data) = c0 * x^(8n) xor crc32(0, data)
        const uint32_t init = crc_in[j] ? multmodp(x2nmodp(host_x2n, n[j], 3), crc_in[j]) : 0u;
        if (n[j] == 0) {
            crcs[j] = crc_in[j];
            continue;
        }
        const uint64_t threads = (n[j] + CRC_SPAN - 1) / CRC_SPAN;
        KTimer kt(c, "crc32");
        hipLaunchKernelGGL(k_crc32, dim3(grid_for(threads, 256)), dim3(256), 0, c->stream, data[j], n[j], init, d + j);
        ST_LAUNCH_CHECK();
    }
    uint32_t *h = (uint32_t *)pinned(c, 4 * (size_t)cnt);
    ST_HIP(hipMemcpyAsync(h, d, 4 * (size_t)cnt, hipMemcpyDeviceToHost, c->stream));
    ST_HIP(hipStreamSynchronize(c->stream));
    for (int j = 0; j < cnt; ++j)
        if (n[j]) crcs[j] = h[j];
}

}  // namespace st

namespace st {

bool sog_texture_cache(const char *name) {
    return !std::strcmp(name, "means_l.webp") || !std::strcmp(name, "means_u.webp");
}

void sog_bundle_dev(st_ctx *c, const st_sog_meta &meta, uint64_t count, const st_sog_textures &tex,
                    uint16_t dos_time, uint16_t dos_date, const uint8_t **out, uint64_t *out_size) {
    // entries in write-sog.ts order (:186-187, :239, :251, :268, :335, :348, :364)
    struct Img {
        const char *name;
        const uint8_t *rgba;
        int w, h;
    };
    std::vector<Img> imgs = {{"means_l.webp", tex.means_l, meta.width, meta.height},
                             {"means_u.webp", tex.means_u, meta.width, meta.height},
                             {"quats.webp", tex.quats, meta.width, meta.height},
                             {"scales.webp", tex.scales, meta.width, meta.height},
                             {"sh0.webp", tex.sh0, meta.width, meta.height}};
    if (meta.sh_bands > 0) {
        imgs.push_back({"shN_centroids.webp", tex.shn_centroids, meta.shn_width, meta.shn_height});
        imgs.push_back({"shN_labels.webp", tex.shn_labels, meta.width, meta.height});
    }
    const int ni = (int)imgs.size();
    std::vector<WebpJob> jobs(ni);
    for (int i = 0; i < ni; ++i) {
        ST_REQUIRE(imgs[i].rgba, ST_ERR_ARG, std::string("sog bundle: texture missing for ") + imgs[i].name);
        const uint64_t cap = webp_max_size(imgs[i].w, imgs[i].h);
        jobs[i] = {imgs[i].rgba, imgs[i].w, imgs[i].h, imgs[i].w * 4,
                   wsT<uint8_t>(c, "sb.o" + std::to_string(i), cap), cap, 0};
        jobs[i].cache = sog_texture_cache(imgs[i].name);
    }
    webp_encode_dev(c, jobs.data(), ni);
    const std::string mj = sog_meta_json(meta, count);
    std::vector<ZipEntry> es;
    for (int i = 0; i < ni; ++i) es.push_back({imgs[i].name, jobs[i].size, 0});
    es.push_back({"meta.json", mj.size(), 0});
    const uint64_t total = zip_size(es);
    ST_REQUIRE(total < (1ull << 32), ST_ERR_ARG, "sog bundle: archive exceeds 4 GiB (no zip64, as the reference)");
    uint8_t *buf = (uint8_t *)archive_buf(c, total);
    std::vector<uint64_t> off(es.size());
    zip_write(es, dos_time, dos_date, buf, off.data());  // offsets; headers rewritten with the CRCs below
    // entry bytes go straight into the pinned archive while the CRC kernels run
    std::memcpy(buf + off[ni], mj.data(), mj.size());
    uint8_t *dmeta = wsT<uint8_t>(c, "sb.meta", mj.size());
    ST_HIP(hipMemcpyAsync(dmeta, buf + off[ni], mj.size(), hipMemcpyHostToDevice, c->stream));
    for (int i = 0; i < ni; ++i)
        if (jobs[i].size)
            ST_HIP(hipMemcpyAsync(buf + off[i], jobs[i].out, jobs[i].size, hipMemcpyDeviceToHost, c->stream));
    std::vector<const uint8_t *> ptrs;
    std::vector<uint64_t> lens;
    for (auto &j : jobs) {
        ptrs.push_back(j.out);
        lens.push_back(j.size);
    }
    ptrs.push_back(dmeta);
    lens.push_back(mj.size());
    std::vector<uint32_t> zero(ptrs.size(), 0), crcs(ptrs.size(), 0);
    crc32_dev(c, ptrs.data(), lens.data(), zero.data(), (int)ptrs.size(), crcs.data());  // synchronises
    for (size_t i = 0; i < es.size(); ++i) es[i].crc = crcs[i];
    zip_write(es, dos_time, dos_date, buf, off.data());
    *out = buf;
    *out_size = total;
}

// ---- writeSog into a file, the archive streamed ------------------------------------------
void sog_file_check(int fd) {
    // the archive is written at absolute offsets (pwrite), so the descriptor must be seekable: a
    // pipe fails here, before any work, instead of with ESPIPE after the step
    ST_REQUIRE(fd >= 0, ST_ERR_ARG, "sog file: bad file descriptor");
    struct stat stt;
    ST_REQUIRE(fstat(fd, &stt) == 0, ST_ERR_ARG, std::string("sog file: fstat failed: ") + std::strerror(errno));
    ST_REQUIRE(S_ISREG(stt.st_mode) || lseek(fd, 0, SEEK_CUR) != (off_t)-1, ST_ERR_ARG,
               "sog file: fd must be a seekable file (a regular file opened for writing)");
    // pwrite on an O_APPEND descriptor ignores the offset (Linux) and a read-only one fails only
    // after the step: both are refused here
    const int fl = fcntl(fd, F_GETFL);
    ST_REQUIRE(fl != -1, ST_ERR_ARG, std::string("sog file: fcntl failed: ") + std::strerror(errno));
    ST_REQUIRE((fl & O_ACCMODE) == O_WRONLY || (fl & O_ACCMODE) == O_RDWR, ST_ERR_ARG,
               "sog file: fd must be open for writing");
    ST_REQUIRE(!(fl & O_APPEND), ST_ERR_ARG, "sog file: fd must not be opened with O_APPEND (writes go at offsets)");
}

void write_at(int fd, const uint8_t *p, uint64_t n, uint64_t off) {
    while (n) {
        const ssize_t w = pwrite(fd, p, n, (off_t)off);
        if (w < 0 && errno == EINTR) continue;
        ST_REQUIRE(w > 0, ST_ERR_ARG, std::string("sog file: write failed: ") + std::strerror(errno));
        p += w;
        n -= (uint64_t)w;
        off += (uint64_t)w;
    }
}

void sog_file_truncate(int fd, uint64_t size) {
    // a file longer than the archive (an earlier, longer content) ends at the archive: zip readers
    // look for the end record from the end of the file
    struct stat stt;
    if (fstat(fd, &stt) == 0 && S_ISREG(stt.st_mode) && (uint64_t)stt.st_size > size)
        ST_REQUIRE(ftruncate(fd, (off_t)size) == 0, ST_ERR_ARG,
                   std::string("sog file: truncate failed: ") + std::strerror(errno));
}

namespace {

struct Img {
    const char *name;
    const uint8_t *rgba;
    int w, h;
};

// entries in order into one pinned block [local header, data, descriptor]...: the images' WebP
// streams and `extra` host entries (meta.json), CRCs on the device; returns the block's bytes
uint64_t stage_entries(st_ctx *c, const std::vector<Img> &imgs, const std::vector<std::string> &extra,
                       const char *const *extra_names, uint16_t dos_time, uint16_t dos_date, const std::string &tag,
                       std::vector<ZipEntry> &es, uint8_t **block) {
    const int ni = (int)imgs.size(), ne = (int)extra.size();
    std::vector<WebpJob> jobs(ni);
    for (int i = 0; i < ni; ++i) {
        ST_REQUIRE(imgs[i].rgba, ST_ERR_ARG, std::string("sog file: texture missing for ") + imgs[i].name);
        const uint64_t cap = webp_max_size(imgs[i].w, imgs[i].h);
        jobs[i] = {imgs[i].rgba, imgs[i].w, imgs[i].h, imgs[i].w * 4, wsT<uint8_t>(c, tag + std::to_string(i), cap),
                   cap, 0};
        jobs[i].cache = sog_texture_cache(imgs[i].name);
    }
    if (ni) webp_encode_dev(c, jobs.data(), ni);
    es.clear();
    for (int i = 0; i < ni; ++i) es.push_back({imgs[i].name, jobs[i].size, 0});
    for (int i = 0; i < ne; ++i) es.push_back({extra_names[i], extra[i].size(), 0});
    uint64_t total = 0;
    for (auto &e : es) total += 30 + e.name.size() + e.size + 16;
    uint8_t *buf = (uint8_t *)pinned_slot(c, tag + "blk", total);
    std::vector<uint64_t> off(es.size());
    uint64_t o = 0;
    for (size_t i = 0; i < es.size(); ++i) {
        o += zip_local(es[i], dos_time, dos_date, buf + o);
        off[i] = o;
        o += es[i].size + 16;
    }
    std::vector<const uint8_t *> ptrs;
    std::vector<uint64_t> lens;
    for (int i = 0; i < ni; ++i) {
        if (jobs[i].size)
            ST_HIP(hipMemcpyAsync(buf + off[i], jobs[i].out, jobs[i].size, hipMemcpyDeviceToHost, c->stream));
        ptrs.push_back(jobs[i].out);
        lens.push_back(jobs[i].size);
    }
    for (int i = 0; i < ne; ++i) {
        std::memcpy(buf + off[ni + i], extra[i].data(), extra[i].size());
        uint8_t *d = wsT<uint8_t>(c, tag + "x" + std::to_string(i), extra[i].size());
        ST_HIP(hipMemcpyAsync(d, buf + off[ni + i], extra[i].size(), hipMemcpyHostToDevice, c->stream));
        ptrs.push_back(d);
        lens.push_back(extra[i].size());
    }
    std::vector<uint32_t> zero(ptrs.size(), 0), crcs(ptrs.size(), 0);
    if (!ptrs.empty()) crc32_dev(c, ptrs.data(), lens.data(), zero.data(), (int)ptrs.size(), crcs.data());  // syncs
    for (size_t i = 0; i < es.size(); ++i) {
        es[i].crc = crcs[i];
        zip_descriptor(es[i], buf + off[i] + es[i].size);
    }
    *block = buf;
    return total;
}
}  // namespace

uint64_t sog_file_dev(st_ctx *c, const st_table *t, int iters, const double *draws, uint64_t ndraws,
                      st_sog_meta *meta, const st_sog_textures *out, int fd, uint16_t dos_time, uint16_t dos_date,
                      uint64_t *file_size) {
    const auto t_call = std::chrono::steady_clock::now();
    sog_file_check(fd);
    // the five textures final before the SH k-means: their entries go to the file from a host
    // thread on the side context (the step's colour k-means, which used it, has joined by then)
    struct Early {
        std::vector<ZipEntry> es;
        uint64_t bytes = 0;
        std::exception_ptr err;
        std::thread th;
        std::chrono::steady_clock::time_point t0, t1, t2;  // hook, early entries staged, written
    } early;
    struct Join {
        Early &e;
        ~Join() {
            if (e.th.joinable()) e.th.join();
        }
    } join{early};
    struct Hook {
        st_ctx *c;
        ~Hook() { c->sog_early = nullptr; }
    } hook{c};
    c->sog_early = [&](st_ctx *cc) {
        st_ctx *aux = cc->aux;
        ST_REQUIRE(aux, ST_ERR_INTERNAL, "sog file: no side context");
        hipEvent_t ev;
        ST_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        ST_HIP(hipEventRecord(ev, cc->stream));
        ST_HIP(hipStreamWaitEvent(aux->stream, ev, 0));
        ST_HIP(hipEventDestroy(ev));
        const std::vector<Img> imgs = {{"means_l.webp", out->means_l, meta->width, meta->height},
                                       {"means_u.webp", out->means_u, meta->width, meta->height},
                                       {"quats.webp", out->quats, meta->width, meta->height},
                                       {"scales.webp", out->scales, meta->width, meta->height},
                                       {"sh0.webp", out->sh0, meta->width, meta->height}};
        early.t0 = std::chrono::steady_clock::now();
        // a speculative host form (st_host_api: run_host_sog) writes nothing before its compare says
        // the host columns are unchanged
        std::function<bool()> verdict = cc->spec_verdict;
        early.th = std::thread([&early, aux, imgs, fd, dos_time, dos_date, verdict] {
            try {
                use_device(aux);
                uint8_t *blk = nullptr;
                early.bytes = stage_entries(aux, imgs, {}, nullptr, dos_time, dos_date, "sf.e", early.es, &blk);
                early.t1 = std::chrono::steady_clock::now();
                if (verdict && !verdict()) throw SpecAbort();
                write_at(fd, blk, early.bytes, 0);
                early.t2 = std::chrono::steady_clock::now();
            } catch (...) {
                early.err = std::current_exception();
            }
        });
    };
    const uint64_t used = sog_dev(c, t, iters, draws, ndraws, meta, out);
    c->sog_early = nullptr;
    const auto t_ret = std::chrono::steady_clock::now();
    if (getenv("ST_DEBUG")) ST_HIP(hipStreamSynchronize(c->stream));
    const auto t_gpu = std::chrono::steady_clock::now();
    ST_REQUIRE(early.th.joinable(), ST_ERR_INTERNAL, "sog file: the early entries never started");
    // shN textures and meta.json on this context while the early entries are written
    std::vector<Img> late;
    if (meta->sh_bands > 0) {
        late.push_back({"shN_centroids.webp", out->shn_centroids, meta->shn_width, meta->shn_height});
        late.push_back({"shN_labels.webp", out->shn_labels, meta->width, meta->height});
    }
    const uint64_t count = t->n;
    const std::vector<std::string> extra = {sog_meta_json(*meta, count)};
    const char *const extra_names[1] = {"meta.json"};
    std::vector<ZipEntry> les;
    uint8_t *lblk = nullptr;
    const uint64_t lbytes = stage_entries(c, late, extra, extra_names, dos_time, dos_date, "sf.l", les, &lblk);
    const auto t3 = std::chrono::steady_clock::now();
    early.th.join();
    if (getenv("ST_DEBUG")) {
        const auto ms = [&](std::chrono::steady_clock::time_point a) {
            return std::chrono::duration<double, std::milli>(a - early.t0).count();
        };
        fprintf(stderr, "[st sog file] after the hook: early entries staged %.1f ms, written %.1f ms; the step "
                "returned %.1f ms, its work done %.1f ms; late entries staged %.1f ms, early thread joined %.1f ms\n",
                ms(early.t1), ms(early.t2), ms(t_ret), ms(t_gpu), ms(t3), ms(std::chrono::steady_clock::now()));
    }
    if (early.err) std::rethrow_exception(early.err);
    spec_gate(c);
    std::vector<ZipEntry> all = early.es;
    all.insert(all.end(), les.begin(), les.end());
    ST_REQUIRE(zip_size(all) < (1ull << 32), ST_ERR_ARG, "sog file: archive exceeds 4 GiB (no zip64, as the reference)");
    const auto t4 = std::chrono::steady_clock::now();
    write_at(fd, lblk, lbytes, early.bytes);
    const auto t5 = std::chrono::steady_clock::now();
    std::vector<uint8_t> cd(zip_central_size(all));
    zip_central(all, dos_time, dos_date, cd.data());
    write_at(fd, cd.data(), cd.size(), early.bytes + lbytes);
    *file_size = early.bytes + lbytes + cd.size();
    sog_file_truncate(fd, *file_size);
    if (getenv("ST_DEBUG")) {
        const auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
            return std::chrono::duration<double, std::milli>(b - a).count();
        };
        fprintf(stderr, "[st sog file] hook %.1f ms after the call; late entries %.1f MB written in %.1f ms; "
                "directory + truncate %.1f ms; the call %.1f ms\n", ms(t_call, early.t0), lbytes / 1e6, ms(t4, t5),
                ms(t5, std::chrono::steady_clock::now()), ms(t_call, std::chrono::steady_clock::now()));
    }
    return used;
}

}  // namespace st

using namespace st;

extern "C" {

uint64_t st_webp_max_size(int32_t width, int32_t height) {
    if (width < 1 || height < 1 || width > 16384 || height > 16384) return 0;
    return webp_max_size(width, height);
}

int st_dev_webp_lossless(st_ctx *c, const uint8_t *rgba, int32_t width, int32_t height, int32_t stride,
                         uint8_t *out, uint64_t cap, uint64_t *size) {
    return guard([&] {
        ST_REQUIRE(c && rgba && out && size, ST_ERR_ARG, "NULL argument");
        use_device(c);
        WebpJob j{rgba, width, height, stride, out, cap, 0};
        webp_encode_dev(c, &j, 1);
        *size = j.size;
    });
}

int st_webp_lossless(st_ctx *c, const uint8_t *rgba, int32_t width, int32_t height, int32_t stride, uint8_t **out,
                     uint64_t *size) {
    return guard([&] {
        ST_REQUIRE(c && rgba && out && size, ST_ERR_ARG, "NULL argument");
        ST_REQUIRE(width >= 1 && height >= 1 && width <= 16384 && height <= 16384 && stride >= width * 4, ST_ERR_ARG,
                   "webp: bad image geometry");
        use_device(c);
        const uint64_t row = (uint64_t)width * 4, bytes = row * height;
        uint8_t *d_in = wsT<uint8_t>(c, "wl.in", bytes);
        ST_HIP(hipMemcpy2DAsync(d_in, row, rgba, stride, row, height, hipMemcpyHostToDevice, c->stream));
        const uint64_t cap = webp_max_size(width, height);
        WebpJob j{d_in, width, height, (int)row, wsT<uint8_t>(c, "wl.out", cap), cap, 0};
        webp_encode_dev(c, &j, 1);
        uint8_t *buf = (uint8_t *)std::malloc(j.size);
        ST_REQUIRE(buf, ST_ERR_NOMEM, "webp: host allocation failed");
        hipError_t e = hipMemcpyAsync(buf, j.out, j.size, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        if (e != hipSuccess) {
            std::free(buf);
            ST_HIP(e);
        }
        *out = buf;
        *size = j.size;
    });
}

int st_dev_crc32(st_ctx *c, const uint8_t *data, uint64_t n, uint32_t crc_in, uint32_t *out) {
    return guard([&] {
        ST_REQUIRE(c && (data || n == 0) && out, ST_ERR_ARG, "NULL argument");
        use_device(c);
        crc32_dev(c, &data, &n, &crc_in, 1, out);
    });
}

int st_dev_sog_bundle(st_ctx *c, const st_sog_meta *meta, uint64_t count, const st_sog_textures *tex,
                      uint16_t dos_time, uint16_t dos_date, uint8_t **out, uint64_t *size) {
    return guard([&] {
        ST_REQUIRE(c && meta && tex && out && size, ST_ERR_ARG, "NULL argument");
        use_device(c);
        const uint8_t *view;
        uint64_t n;
        sog_bundle_dev(c, *meta, count, *tex, dos_time, dos_date, &view, &n);
        uint8_t *buf = (uint8_t *)std::malloc(n);
        ST_REQUIRE(buf, ST_ERR_NOMEM, "sog bundle: host allocation failed");
        std::memcpy(buf, view, n);
        *out = buf;
        *size = n;
    });
}

int st_dev_sog_bundle_view(st_ctx *c, const st_sog_meta *meta, uint64_t count, const st_sog_textures *tex,
                           uint16_t dos_time, uint16_t dos_date, const uint8_t **out, uint64_t *size) {
    return guard([&] {
        ST_REQUIRE(c && meta && tex && out && size, ST_ERR_ARG, "NULL argument");
        use_device(c);
        sog_bundle_dev(c, *meta, count, *tex, dos_time, dos_date, out, size);
    });
}

}  // extern "C"
