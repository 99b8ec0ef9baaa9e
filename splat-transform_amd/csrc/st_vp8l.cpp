// st_vp8l.cpp -- VP8L prefix codes and header bits (host; see st_vp8l.h).
//
// Bitstream layout follows the WebP lossless format (RFC 9649): signature 0x2f,
// 14-bit width-1 / height-1, alpha hint, version 0; transforms; colour-cache bit;
// meta-prefix bit (main image only); five prefix codes (green + length prefixes,
// red, blue, alpha, distance); the entropy-coded pixels.
#include "st_vp8l.h"

#include <algorithm>
#include <cmath>
#include <stdexcept>

namespace st {
namespace vp8l {

void BitWriter::put(uint32_t v, int n) {
    if (n == 0) return;
    acc |= (uint64_t)(v & ((n == 32) ? 0xffffffffu : ((1u << n) - 1))) << nacc;
    nacc += n;
    nbits += (uint64_t)n;
    while (nacc >= 8) {
        buf.push_back((uint8_t)acc);
        acc >>= 8;
        nacc -= 8;
    }
}

std::vector<uint8_t> BitWriter::bytes() const {
    std::vector<uint8_t> b = buf;
    if (nacc) b.push_back((uint8_t)acc);
    return b;
}

// Huffman over the used symbols with counts raised to at least `floor`; depths out.  Two-queue
// construction: the leaves sorted once by (weight, index), the merged nodes appended in
// non-decreasing weight order; a leaf wins a weight tie (deterministic)
static int huffman_depths(const std::vector<std::pair<uint64_t, int>> &used, uint64_t floor_,
                          std::vector<int> &depth) {
    const int m = (int)used.size();
    std::vector<std::pair<uint64_t, int>> leaf(m);
    for (int i = 0; i < m; ++i) leaf[i] = {std::max(used[i].first, floor_), i};
    std::sort(leaf.begin(), leaf.end());
    std::vector<uint64_t> iw;  // merged nodes' weights (node id m + index)
    iw.reserve(m);
    std::vector<int> parent(2 * m, -1);
    int li = 0, ii = 0;
    auto take = [&]() {
        if (li < m && (ii >= (int)iw.size() || leaf[li].first <= iw[ii])) {
            const auto &l = leaf[li++];
            return std::make_pair(l.first, l.second);
        }
        const int id = m + ii;
        return std::make_pair(iw[ii++], id);
    };
    for (int k = 0; k < m - 1; ++k) {
        const auto a = take(), b = take();
        parent[a.second] = m + k;
        parent[b.second] = m + k;
        iw.push_back(a.first + b.first);
    }
    // depths top-down: merged nodes are numbered in creation order, so a parent has a larger id
    std::vector<int> d(2 * m, 0);
    int maxd = 0;
    for (int v = 2 * m - 3; v >= 0; --v) d[v] = d[parent[v]] + 1;
    depth.assign(m, 0);
    for (int i = 0; i < m; ++i) {
        depth[i] = d[i];
        maxd = std::max(maxd, d[i]);
    }
    return maxd;
}

void huffman_lengths(const uint64_t *counts, int n, int limit, uint8_t *len) {
    std::vector<std::pair<uint64_t, int>> used;
    for (int s = 0; s < n; ++s) {
        len[s] = 0;
        if (counts[s]) used.push_back({counts[s], s});
    }
    if (used.empty()) return;
    if (used.size() == 1) {
        len[used[0].second] = 1;
        return;
    }
    // raising small counts flattens the tree until it fits the length limit (the
    // result is still a full binary tree, i.e. a complete code)
    std::vector<int> depth;
    if (huffman_depths(used, 1, depth) > limit) {
        // a floor of total / 2^(limit - 1) always fits the limit; start a few doublings below it
        uint64_t total = 0;
        for (auto &u : used) total += u.first;
        uint64_t floor_ = std::max<uint64_t>(2, total >> (limit + 2));
        while (huffman_depths(used, floor_, depth) > limit) floor_ *= 2;
    }
    for (size_t i = 0; i < used.size(); ++i) len[used[i].second] = (uint8_t)depth[i];
}

// canonical codes (shorter first, ascending symbol within a length), bit-reversed
static void canonical(const uint8_t *len, int n, uint16_t *rev) {
    int bl[kMaxCodeLen + 2] = {0};
    for (int s = 0; s < n; ++s) bl[len[s]]++;
    bl[0] = 0;
    uint32_t next[kMaxCodeLen + 2] = {0};
    uint32_t code = 0;
    for (int b = 1; b <= kMaxCodeLen + 1; ++b) {
        code = (code + bl[b - 1]) << 1;
        next[b] = code;
    }
    for (int s = 0; s < n; ++s) {
        rev[s] = 0;
        const int l = len[s];
        if (!l) continue;
        const uint32_t c = next[l]++;
        uint32_t r = 0;
        for (int i = 0; i < l; ++i) r |= ((c >> i) & 1u) << (l - 1 - i);
        rev[s] = (uint16_t)r;
    }
}

static const int kCodeLengthOrder[19] = {17, 18, 0, 1, 2, 3, 4, 5, 16, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15};

Code write_code(BitWriter &bw, const uint64_t *counts, int alphabet) {
    Code c;
    c.len.assign(alphabet, 0);
    c.rev.assign(alphabet, 0);
    std::vector<int> used;
    for (int s = 0; s < alphabet; ++s)
        if (counts[s]) used.push_back(s);
    if (used.empty()) used.push_back(0);  // an unused alphabet: one zero-bit symbol
    if (used.size() <= 2 && used.back() < 256) {
        // simple code: 1 or 2 symbols, lengths 0 or 1
        bw.put(1, 1);
        bw.put((uint32_t)used.size() - 1, 1);
        if (used[0] < 2) {
            bw.put(0, 1);
            bw.put((uint32_t)used[0], 1);
        } else {
            bw.put(1, 1);
            bw.put((uint32_t)used[0], 8);
        }
        if (used.size() == 2) {
            bw.put((uint32_t)used[1], 8);
            c.len[used[0]] = 1;
            c.len[used[1]] = 1;
            c.rev[used[1]] = 1;  // ascending symbols: used[0] < used[1] gets code 0
        }
        return c;
    }
    // normal code
    huffman_lengths(counts, alphabet, kMaxCodeLen, c.len.data());
    canonical(c.len.data(), alphabet, c.rev.data());
    // run-length tokens over the code lengths: 0..15 literal, 16 repeat previous
    // non-zero 3..6, 17 zeros 3..10, 18 zeros 11..138
    struct Tok {
        uint8_t sym, extra_bits;
        uint8_t extra;
    };
    std::vector<Tok> toks;
    for (int i = 0; i < alphabet;) {
        const int v = c.len[i];
        int run = 1;
        while (i + run < alphabet && c.len[i + run] == v) ++run;
        i += run;
        if (v == 0) {
            while (run > 0) {
                if (run >= 11) {
                    const int r = std::min(run, 138);
                    toks.push_back({18, 7, (uint8_t)(r - 11)});
                    run -= r;
                } else if (run >= 3) {
                    const int r = std::min(run, 10);
                    toks.push_back({17, 3, (uint8_t)(r - 3)});
                    run -= r;
                } else {
                    toks.push_back({0, 0, 0});
                    --run;
                }
            }
        } else {
            toks.push_back({(uint8_t)v, 0, 0});
            --run;
            while (run >= 3) {
                const int r = std::min(run, 6);
                toks.push_back({16, 2, (uint8_t)(r - 3)});
                run -= r;
            }
            while (run-- > 0) toks.push_back({(uint8_t)v, 0, 0});
        }
    }
    uint64_t tc[19] = {0};
    for (auto &t : toks) tc[t.sym]++;
    uint8_t cl[19];
    huffman_lengths(tc, 19, 7, cl);
    uint16_t crev[19];
    canonical(cl, 19, crev);
    int nused = 0;
    for (int s = 0; s < 19; ++s) nused += cl[s] != 0;
    int ncl = 4;
    for (int i = 0; i < 19; ++i)
        if (cl[kCodeLengthOrder[i]]) ncl = std::max(ncl, i + 1);
    bw.put(0, 1);  // normal code
    bw.put((uint32_t)(ncl - 4), 4);
    for (int i = 0; i < ncl; ++i) bw.put(cl[kCodeLengthOrder[i]], 3);
    bw.put(0, 1);  // max_symbol = alphabet size
    for (auto &t : toks) {
        // a one-symbol code-length code is read with zero bits
        if (nused > 1) bw.put(crev[t.sym], cl[t.sym]);
        bw.put(t.extra, t.extra_bits);
    }
    return c;
}

// a sub-image (predictor modes, entropy image): green = the value, no colour cache
static void write_subimage(BitWriter &bw, const uint8_t *v, size_t n) {
    std::vector<uint64_t> g(kGreenAlphabet, 0), zero(256, 0), dist(kDistAlphabet, 0);
    for (size_t i = 0; i < n; ++i) g[v[i]]++;
    zero[0] = 1;
    bw.put(0, 1);  // no colour cache
    Code cg = write_code(bw, g.data(), kGreenAlphabet);
    write_code(bw, zero.data(), 256);  // red 0
    write_code(bw, zero.data(), 256);  // blue 0
    write_code(bw, zero.data(), 256);  // alpha 0
    write_code(bw, dist.data(), kDistAlphabet);
    for (size_t i = 0; i < n; ++i) bw.put(cg.rev[v[i]], cg.len[v[i]]);
}

void build_header(int width, int height, bool alpha_used, const uint32_t *hist, int ngroups, const uint8_t *groups,
                  int group_bits, const uint8_t *modes, int cache_bits, Header &out) {
    if (width < 1 || height < 1 || width > 16384 || height > 16384)
        throw std::invalid_argument("vp8l: image size out of range");
    if (cache_bits != 0 && (cache_bits < kMinCacheBits || cache_bits > kMaxCacheBits))
        throw std::invalid_argument("vp8l: colour cache bits out of range");
    if (ngroups < 1 || ngroups > 256 || (ngroups > 1 && (group_bits < 2 || group_bits > 9)))
        throw std::invalid_argument("vp8l: prefix-code groups out of range");
    BitWriter &bw = out.bw;
    bw.put(0x2f, 8);
    bw.put((uint32_t)(width - 1), 14);
    bw.put((uint32_t)(height - 1), 14);
    bw.put(alpha_used ? 1 : 0, 1);
    bw.put(0, 3);
    // predictor transform with its sub-image (entropy-coded image: green = mode)
    bw.put(1, 1);
    bw.put(0, 2);
    bw.put(kPredBits - 2, 3);
    const int bw_ = (width + (1 << kPredBits) - 1) >> kPredBits;
    const int bh_ = (height + (1 << kPredBits) - 1) >> kPredBits;
    write_subimage(bw, modes, (size_t)bw_ * bh_);
    bw.put(0, 1);  // no more transforms
    // main image
    if (cache_bits) {
        bw.put(1, 1);
        bw.put((uint32_t)cache_bits, 4);
    } else {
        bw.put(0, 1);  // no colour cache
    }
    if (ngroups > 1) {  // meta prefix codes: the entropy image (green = group)
        bw.put(1, 1);
        bw.put((uint32_t)(group_bits - 2), 3);
        const int gw = (width + (1 << group_bits) - 1) >> group_bits;
        const int gh = (height + (1 << group_bits) - 1) >> group_bits;
        write_subimage(bw, groups, (size_t)gw * gh);
    } else {
        bw.put(0, 1);  // one prefix-code group
    }
    out.tab.assign((size_t)ngroups * kTabSize, 0);
    const int off[5] = {kOffG, kOffR, kOffB, kOffA, kOffD};
    const int size[5] = {kGreenAlphabet + (cache_bits ? 1 << cache_bits : 0), 256, 256, 256, kDistAlphabet};
    for (int g = 0; g < ngroups; ++g)
        for (int ch = 0; ch < 5; ++ch) {
            std::vector<uint64_t> cnt(size[ch], 0);
            for (int s = 0; s < size[ch]; ++s) cnt[s] = hist[(size_t)g * kTabSize + off[ch] + s];
            Code code = write_code(bw, cnt.data(), size[ch]);
            for (int s = 0; s < size[ch]; ++s)
                out.tab[(size_t)g * kTabSize + off[ch] + s] = ((uint32_t)code.len[s] << 16) | code.rev[s];
        }
}

double literal_bits(const uint32_t *hist) {
    const int off[4] = {kOffG, kOffR, kOffB, kOffA};
    double bits = 0;
    for (int ch = 0; ch < 4; ++ch) {
        double n = 0;
        for (int s = 0; s < 256; ++s) n += hist[off[ch] + s];
        for (int s = 0; s < 256; ++s)
            if (hist[off[ch] + s]) bits -= hist[off[ch] + s] * std::log2(hist[off[ch] + s] / n);
    }
    return bits;
}

// bits of one prefix code: its description plus the symbols it codes
static double code_bits(const std::vector<uint64_t> &c) {
    BitWriter scratch;
    const Code code = write_code(scratch, c.data(), (int)c.size());
    double b = (double)scratch.nbits;
    for (size_t s = 0; s < c.size(); ++s) b += (double)c[s] * code.len[s];
    return b;
}

static double shannon(const uint64_t *c, int n) {
    double t = 0, bits = 0;
    for (int s = 0; s < n; ++s) t += (double)c[s];
    for (int s = 0; s < n; ++s)
        if (c[s]) bits -= (double)c[s] * std::log2((double)c[s] / t);
    return bits;
}

int choose_cache_bits(const uint32_t *hist, const uint32_t *hitlit, const uint32_t *cidx) {
    const int off[4] = {kOffG, kOffR, kOffB, kOffA};
    // per candidate: the green alphabet (literals, length prefixes, cache indices) and the red,
    // blue, alpha literals left after the hits of the sizes <= bits
    struct Cand {
        int bits;
        std::vector<uint64_t> g, rba;
        double est;
    };
    std::vector<Cand> cand;
    std::vector<uint64_t> lit(4 * 256);
    for (int ch = 0; ch < 4; ++ch)
        for (int v = 0; v < 256; ++v) lit[ch * 256 + v] = hist[off[ch] + v];
    for (int bits = 0; bits <= kMaxCacheBits; bits = bits ? bits + 1 : kMinCacheBits) {
        if (bits) {
            const uint32_t *h = hitlit + (size_t)(bits - kMinCacheBits) * 1024;
            for (int i = 0; i < 1024; ++i) lit[i] -= h[i];
        }
        Cand c{bits, std::vector<uint64_t>(lit.begin(), lit.begin() + 256),
               std::vector<uint64_t>(lit.begin() + 256, lit.end()), 0.0};
        for (int s = 256; s < kGreenAlphabet; ++s) c.g.push_back(hist[kOffG + s]);
        int used = 0;
        if (bits)
            for (int s = 0; s < (1 << bits); ++s) {
                c.g.push_back(cidx[cache_off(bits) + s]);
                used += cidx[cache_off(bits) + s] != 0;
            }
        // Shannon bits plus ~4 bits per used cache symbol's code length: the preselection
        c.est = shannon(c.g.data(), (int)c.g.size()) + 4.0 * used;
        for (int ch = 0; ch < 3; ++ch) c.est += shannon(c.rba.data() + ch * 256, 256);
        cand.push_back(std::move(c));
    }
    // the coded size (descriptions + symbols) of no cache and the two best estimates, when the
    // estimates are within 2% of each other (otherwise the estimate decides)
    std::vector<int> order(cand.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = (int)i;
    std::stable_sort(order.begin() + 1, order.end(), [&](int a, int b) { return cand[a].est < cand[b].est; });
    const double e0 = cand[0].est, e1 = cand[order[1]].est;
    if (e1 < 0.98 * e0) return cand[order[1]].bits;
    if (e1 > 1.02 * e0) return 0;
    int best = 0;
    double bc = 0;
    for (int k = 0; k < 3 && k < (int)order.size(); ++k) {
        const Cand &c = cand[order[k]];
        double b = code_bits(c.g);
        for (int ch = 0; ch < 3; ++ch)
            b += code_bits(std::vector<uint64_t>(c.rba.begin() + ch * 256, c.rba.begin() + ch * 256 + 256));
        if (k == 0 || b < bc) {
            bc = b;
            best = c.bits;
        }
    }
    return best;
}

}  // namespace vp8l
}  // namespace st
