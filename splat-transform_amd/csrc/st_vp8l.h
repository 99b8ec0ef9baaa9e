// st_vp8l.h -- host side of the WebP lossless (VP8L) encoder: prefix-code
// construction and the bitstream header.  The per-pixel work (predictor choice,
// residuals, histograms, the entropy-coded pixel stream) runs on the device
// (st_webp.hip); the host turns four 256-bin histograms into canonical prefix
// codes and writes the few hundred header bits in front of the pixel stream.
//
// Replaces the reference's WebPEncodeLosslessRGBA (lib/webp_encode.c:19-29,
// called from utils/webp.ts:19-41 by write-sog.ts:120-140).  Parity is at the
// decoded-RGBA level: any valid lossless VP8L stream of the same
// pixels is a drop-in; the byte stream itself differs from libwebp's.
#pragma once

#include <cstdint>
#include <vector>

namespace st {
namespace vp8l {

constexpr int kPredBits = 4;           // predictor blocks of 16 x 16 pixels
constexpr int kGreenAlphabet = 280;    // 256 literals + 24 length prefixes (no colour cache)
constexpr int kDistAlphabet = 40;
constexpr int kMaxCodeLen = 15;
// colour cache (RFC 9649 5.2.2): the candidate sizes are 2^4 .. 2^10 entries; a pixel whose colour
// sits in the cache at (0x1e35a7bd * argb) >> (32 - bits) is coded as one green symbol 280 + index
constexpr int kMinCacheBits = 4, kMaxCacheBits = 10;
constexpr int kCacheLevels = kMaxCacheBits - kMinCacheBits + 1;
constexpr int kCacheSlots = (2 << kMaxCacheBits) - (1 << kMinCacheBits);  // all levels' slots: 2,032
constexpr int cache_off(int bits) { return (1 << bits) - (1 << kMinCacheBits); }  // level's first slot
constexpr uint32_t kCacheMul = 0x1e35a7bdu;
constexpr int kGreenMax = kGreenAlphabet + (1 << kMaxCacheBits);
// the device histogram / code-table layout: G (280 + the cache symbols: literals, length
// prefixes, cache indices), R, B, A (256 each), distance (40)
constexpr int kOffG = 0, kOffR = kGreenMax, kOffB = kOffR + 256, kOffA = kOffB + 256, kOffD = kOffA + 256;
constexpr int kTabSize = kOffD + kDistAlphabet;

// LSB-first bit writer (the VP8L bit order)
struct BitWriter {
    std::vector<uint8_t> buf;
    uint64_t acc = 0;
    int nacc = 0;
    uint64_t nbits = 0;
    void put(uint32_t v, int n);
    // the bytes written so far, the last one partial (zero high bits)
    std::vector<uint8_t> bytes() const;
};

// one prefix code: per symbol the emitted length (0 for a one-symbol code) and the
// canonical code with its bits reversed (VP8L reads codes MSB-first from an LSB-first stream)
struct Code {
    std::vector<uint8_t> len;
    std::vector<uint16_t> rev;
};

// length-limited Huffman code lengths for counts[0..n) (a complete code when >= 2 symbols)
void huffman_lengths(const uint64_t *counts, int n, int limit, uint8_t *len);

// build the code for counts[0..alphabet) and append its description to bw
// (simple code for <= 2 used symbols below 256, normal code otherwise)
Code write_code(BitWriter &bw, const uint64_t *counts, int alphabet);

// The header bits of one image: everything before the main image's pixel
// stream (VP8L signature, size, predictor transform with its entropy-coded
// sub-image, colour-cache and meta-code flags, the entropy image when there are
// several prefix-code groups, then five prefix codes per group).
// hist: ngroups x kTabSize symbol histograms (each in the kOff* layout: G with the
// length prefixes, R, B, A, distance); groups (ngroups > 1): the entropy image, one
// group index per 2^group_bits-square block (row-major); modes: the predictor
// sub-image (one byte per 16 x 16 block, row-major).
// tab (out): ngroups x kTabSize device table entries (len << 16 | reversed code).
struct Header {
    BitWriter bw;
    std::vector<uint32_t> tab;
};
// cache_bits: 0 (no colour cache) or kMinCacheBits..kMaxCacheBits (green alphabet 280 + 2^bits)
void build_header(int width, int height, bool alpha_used, const uint32_t *hist, int ngroups, const uint8_t *groups,
                  int group_bits, const uint8_t *modes, int cache_bits, Header &out);
// Shannon bits of the literal symbols of a kTabSize histogram (channels G, R, B, A): the
// cost estimate that decides between predictors for a whole image
double literal_bits(const uint32_t *hist);
// The colour-cache size of an image, from one pass over its tokens: hist = the kTabSize
// histogram without a cache (all prefix-code groups added); hitlit = kCacheLevels x 1,024 counts:
// level l holds the G, R, B, A values (256 each) of the literals whose smallest hitting cache is
// 2^(kMinCacheBits + l) (a literal that hits a cache also hits every larger one); cidx =
// kCacheSlots counts of the hitting literals' cache indices per level (cache_off layout).
// Returns 0 or the bits whose coded size is the smallest (prefix-code descriptions plus coded
// symbols of the green, red, blue and alpha alphabets, as one prefix-code group would code them),
// among no cache and the two sizes with the smallest Shannon estimates (the estimates alone
// decide when the best cache size and no cache are more than 2% apart).
int choose_cache_bits(const uint32_t *hist, const uint32_t *hitlit, const uint32_t *cidx);

}  // namespace vp8l
}  // namespace st
