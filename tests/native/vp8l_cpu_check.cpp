// TEST INFRASTRUCTURE ONLY: a scalar host emulation of the device VP8L kernels
// (st_webp.hip: predictor choice, residuals, histograms, pixel stream) around the
// product's own header/prefix-code builder (st_vp8l.cpp), so the bitstream format
// can be checked on a machine without a GPU (tests/test_webp_cpu.py decodes the
// output with Pillow/libwebp).  Never linked into libsplat_hip.
//
//   vp8l_cpu_check in.rgba W H out.webp [cache_bits]   (cache_bits: -1 = choose, 0 = none, 4..10)
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../splat-transform_amd/csrc/st_vp8l.h"

using namespace st::vp8l;

static uint32_t ch(uint32_t v, int c) { return (v >> (8 * c)) & 0xffu; }
static uint32_t avg2(uint32_t a, uint32_t b) { return (((a ^ b) & 0xfefefefeu) >> 1) + (a & b); }
static uint32_t clamp_full(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r = 0;
    for (int k = 0; k < 4; ++k) {
        int v = (int)ch(a, k) + (int)ch(b, k) - (int)ch(c, k);
        v = v < 0 ? 0 : (v > 255 ? 255 : v);
        r |= (uint32_t)v << (8 * k);
    }
    return r;
}
static uint32_t clamp_half(uint32_t a, uint32_t b) {
    uint32_t r = 0;
    for (int k = 0; k < 4; ++k) {
        const int x = (int)ch(a, k), y = (int)ch(b, k);
        int v = x + (x - y) / 2;
        v = v < 0 ? 0 : (v > 255 ? 255 : v);
        r |= (uint32_t)v << (8 * k);
    }
    return r;
}
static uint32_t sel(uint32_t L, uint32_t T, uint32_t TL) {
    int pl = 0, pt = 0;
    for (int k = 0; k < 4; ++k) {
        pl += abs((int)ch(T, k) - (int)ch(TL, k));
        pt += abs((int)ch(L, k) - (int)ch(TL, k));
    }
    return pl < pt ? L : T;
}
static uint32_t pred(int m, uint32_t L, uint32_t T, uint32_t TL, uint32_t TR) {
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
        case 11: return sel(L, T, TL);
        case 12: return clamp_full(L, T, TL);
        default: return clamp_half(avg2(L, T), TL);
    }
}
static uint32_t sub(uint32_t a, uint32_t b) {
    uint32_t r = 0;
    for (int k = 0; k < 4; ++k) r |= ((ch(a, k) - ch(b, k)) & 0xffu) << (8 * k);
    return r;
}

int main(int argc, char **argv) {
    if (argc != 5 && argc != 6) return 2;
    const int w = atoi(argv[2]), h = atoi(argv[3]);
    const int force_cb = argc == 6 ? atoi(argv[5]) : -1;
    std::vector<uint8_t> rgba((size_t)w * h * 4);
    FILE *f = fopen(argv[1], "rb");
    if (!f || fread(rgba.data(), 1, rgba.size(), f) != rgba.size()) return 3;
    fclose(f);
    std::vector<uint32_t> argb((size_t)w * h);
    bool alpha = false;
    for (size_t i = 0; i < argb.size(); ++i) {
        const uint8_t *p = &rgba[i * 4];
        argb[i] = ((uint32_t)p[3] << 24) | ((uint32_t)p[0] << 16) | ((uint32_t)p[1] << 8) | p[2];
        alpha = alpha || p[3] != 255;
    }
    auto at = [&](int x, int y) { return argb[(size_t)y * w + x]; };
    const int B = 1 << kPredBits, bw = (w + B - 1) / B, bh = (h + B - 1) / B;
    std::vector<uint8_t> modes((size_t)bw * bh);
    std::vector<uint32_t> res((size_t)w * h);
    for (int by = 0; by < bh; ++by)
        for (int bx = 0; bx < bw; ++bx) {
            uint64_t cost[14] = {0};
            for (int y = by * B; y < std::min(h, by * B + B); ++y)
                for (int x = bx * B; x < std::min(w, bx * B + B); ++x) {
                    if (x == 0 || y == 0) continue;
                    const uint32_t TR = (x + 1 < w) ? at(x + 1, y - 1) : at(0, y);
                    for (int m = 0; m < 14; ++m) {
                        const uint32_t r = sub(at(x, y), pred(m, at(x - 1, y), at(x, y - 1), at(x - 1, y - 1), TR));
                        for (int k = 0; k < 4; ++k) cost[m] += ch(r, k) < 128 ? ch(r, k) : 256 - ch(r, k);
                    }
                }
            int best = 0;
            for (int m = 1; m < 14; ++m)
                if (cost[m] < cost[best]) best = m;
            modes[(size_t)by * bw + bx] = (uint8_t)best;
        }
    // the device encoder's choices, restated: residuals of the chosen predictors; tokens (runs of
    // >= 3 residuals equal to their left neighbour inside each 4,096-pixel group become copies at
    // distance code 2); blocks of 32 x 32 holding a literal alpha residual form prefix-code group 1;
    // when the pixels themselves (predictor 0) take fewer literal bits, everything is redone with
    // predictor 0
    auto prefix_of = [](uint32_t v, uint32_t &pfx, uint32_t &ne, uint32_t &ex) {
        if (v <= 4) {
            pfx = v - 1, ne = 0, ex = 0;
            return;
        }
        const uint32_t d = v - 1;
        uint32_t hb = 31 - __builtin_clz(d);
        ne = hb - 1;
        ex = d & ((1u << ne) - 1);
        pfx = 2 * hb + ((d >> (hb - 1)) & 1u);
    };
    const size_t npix = res.size();
    const int GB = 5, gw = (w + (1 << GB) - 1) >> GB, gh = (h + (1 << GB) - 1) >> GB;
    std::vector<uint32_t> tok(npix, 0);  // 0 literal, 0xffff covered, else copy length
    std::vector<uint8_t> gfl((size_t)gw * gh, 0);
    std::vector<uint32_t> hist(2 * kTabSize, 0), raw(kTabSize, 0);
    auto encode_pass = [&](bool force0) {
        for (int y = 0; y < h; ++y)
            for (int x = 0; x < w; ++x) {
                uint32_t p;
                if (y == 0)
                    p = x == 0 ? 0xff000000u : at(x - 1, y);
                else if (x == 0)
                    p = at(x, y - 1);
                else {
                    const uint32_t TR = (x + 1 < w) ? at(x + 1, y - 1) : at(0, y);
                    const int m = force0 ? 0 : modes[(size_t)(y / B) * bw + x / B];
                    p = pred(m, at(x - 1, y), at(x, y - 1), at(x - 1, y - 1), TR);
                }
                res[(size_t)y * w + x] = sub(at(x, y), p);
            }
        std::fill(tok.begin(), tok.end(), 0u);
        for (size_t g0 = 0; g0 < npix; g0 += 4096) {
            const size_t g1 = std::min(npix, g0 + 4096);
            for (size_t i = g0; i < g1;) {
                if (i > 0 && res[i] == res[i - 1]) {
                    size_t j = i;
                    while (j < g1 && res[j] == res[j - 1]) ++j;
                    if (j - i >= 3) {
                        tok[i] = (uint32_t)(j - i);
                        for (size_t q = i + 1; q < j; ++q) tok[q] = 0xffff;
                    }
                    i = j;
                } else {
                    ++i;
                }
            }
        }
        std::fill(gfl.begin(), gfl.end(), 0);
        for (size_t i = 0; i < npix; ++i)
            if (tok[i] == 0 && (res[i] >> 24) != 0) gfl[(i / w >> GB) * gw + ((i % w) >> GB)] = 1;
        std::fill(hist.begin(), hist.end(), 0u);
        std::fill(raw.begin(), raw.end(), 0u);
        for (size_t i = 0; i < npix; ++i) {
            const uint32_t v = sub(argb[i], 0xff000000u);
            raw[kOffG + ch(v, 1)]++, raw[kOffR + ch(v, 2)]++, raw[kOffB + ch(v, 0)]++, raw[kOffA + ch(v, 3)]++;
            if (tok[i] == 0xffff) continue;
            uint32_t *H = hist.data() + (size_t)gfl[(i / w >> GB) * gw + ((i % w) >> GB)] * kTabSize;
            if (tok[i]) {
                uint32_t pfx, ne, ex;
                prefix_of(tok[i], pfx, ne, ex);
                H[kOffG + 256 + pfx]++;
                H[kOffD + 1]++;
                continue;
            }
            const uint32_t r = res[i];
            H[kOffG + ch(r, 1)]++, H[kOffR + ch(r, 2)]++, H[kOffB + ch(r, 0)]++, H[kOffA + ch(r, 3)]++;
        }
    };
    encode_pass(false);
    if (literal_bits(raw.data()) < 0.995 * (literal_bits(hist.data()) + literal_bits(hist.data() + kTabSize))) {
        std::fill(modes.begin(), modes.end(), 0);
        encode_pass(true);
    }
    // colour cache (the device's k_cc_* kernels restated): bit l of hit[i] when the last earlier
    // pixel with the same index in a 2^(4 + l)-entry cache has the same colour (none: a miss)
    std::vector<uint8_t> hit(npix, 0);
    for (int l = 0; l < kCacheLevels; ++l) {
        const int bits = kMinCacheBits + l;
        std::vector<int64_t> last((size_t)1 << bits, -1);
        for (size_t i = 0; i < npix; ++i) {
            const uint32_t s = (res[i] * kCacheMul) >> (32 - bits);
            if (last[s] >= 0 && res[last[s]] == res[i]) hit[i] |= (uint8_t)(1u << l);
            last[s] = (int64_t)i;
        }
    }
    std::vector<uint32_t> hitlit(kCacheLevels * 1024, 0), cidx(kCacheSlots, 0), merged(kTabSize);
    for (size_t i = 0; i < npix; ++i) {
        if (tok[i] != 0 || !hit[i]) continue;
        const int l0 = __builtin_ctz(hit[i]);
        const uint32_t r = res[i];
        uint32_t *hl = hitlit.data() + (size_t)l0 * 1024;
        hl[ch(r, 1)]++, hl[256 + ch(r, 2)]++, hl[512 + ch(r, 0)]++, hl[768 + ch(r, 3)]++;
        for (int l = l0; l < kCacheLevels; ++l) {
            const int bits = kMinCacheBits + l;
            cidx[cache_off(bits) + ((r * kCacheMul) >> (32 - bits))]++;
        }
    }
    for (int q = 0; q < kTabSize; ++q) merged[q] = hist[q] + hist[kTabSize + q];
    const int cb = force_cb >= 0 ? force_cb : choose_cache_bits(merged.data(), hitlit.data(), cidx.data());
    auto cache_hit = [&](size_t i) { return cb && tok[i] == 0 && ((hit[i] >> (cb - kMinCacheBits)) & 1); };
    if (cb) {  // the histograms again: a hitting literal is one green symbol 280 + its index
        for (size_t i = 0; i < npix; ++i) {
            if (!cache_hit(i)) continue;
            const uint32_t r = res[i];
            uint32_t *H = hist.data() + (size_t)gfl[(i / w >> GB) * gw + ((i % w) >> GB)] * kTabSize;
            H[kOffG + ch(r, 1)]--, H[kOffR + ch(r, 2)]--, H[kOffB + ch(r, 0)]--, H[kOffA + ch(r, 3)]--;
            H[kOffG + kGreenAlphabet + ((r * kCacheMul) >> (32 - cb))]++;
        }
        for (int q = 0; q < kTabSize; ++q) merged[q] = hist[q] + hist[kTabSize + q];
    }
    fprintf(stderr, "cache_bits %d\n", cb);
    int ngroups = 1;
    for (uint8_t f : gfl) ngroups = f ? 2 : ngroups;
    Header hd;
    if (ngroups == 2)
        build_header(w, h, alpha, hist.data(), 2, gfl.data(), GB, modes.data(), cb, hd);
    else
        build_header(w, h, alpha, merged.data(), 1, gfl.data(), GB, modes.data(), cb, hd);
    BitWriter &bw_ = hd.bw;
    for (size_t i = 0; i < npix; ++i) {
        const uint32_t r = res[i];
        if (tok[i] == 0xffff) continue;
        const uint32_t *T = hd.tab.data() + (ngroups == 2 ? (size_t)gfl[(i / w >> GB) * gw + ((i % w) >> GB)] : 0) * kTabSize;
        if (tok[i]) {
            uint32_t pfx, ne, ex;
            prefix_of(tok[i], pfx, ne, ex);
            const uint32_t eg = T[kOffG + 256 + pfx], ed = T[kOffD + 1];
            bw_.put(eg & 0xffffu, (int)(eg >> 16));
            bw_.put(ex, (int)ne);
            bw_.put(ed & 0xffffu, (int)(ed >> 16));
            continue;
        }
        if (cache_hit(i)) {
            const uint32_t e = T[kOffG + kGreenAlphabet + ((r * kCacheMul) >> (32 - cb))];
            bw_.put(e & 0xffffu, (int)(e >> 16));
            continue;
        }
        const uint32_t e[4] = {T[kOffG + ch(r, 1)], T[kOffR + ch(r, 2)], T[kOffB + ch(r, 0)], T[kOffA + ch(r, 3)]};
        for (int k = 0; k < 4; ++k) bw_.put(e[k] & 0xffffu, (int)(e[k] >> 16));
    }
    std::vector<uint8_t> body = bw_.bytes();
    const uint32_t vsz = (uint32_t)body.size(), pad = vsz & 1, riff = 4 + 8 + vsz + pad;
    FILE *o = fopen(argv[4], "wb");
    fwrite("RIFF", 1, 4, o);
    fwrite(&riff, 4, 1, o);
    fwrite("WEBPVP8L", 1, 8, o);
    fwrite(&vsz, 4, 1, o);
    fwrite(body.data(), 1, body.size(), o);
    if (pad) fputc(0, o);
    fclose(o);
    return 0;
}
