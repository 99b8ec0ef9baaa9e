// st_ply.hip -- PLY ingest and the compressed-PLY reader on the device (SURVEY.md 8f
// ranks 2 and 4).
//
//   header         readers/read-ply.ts:111-137 (search for "\nend_header\n" within
//                  128 KiB), parseHeader :54-110 (host; same accepted grammar and errors)
//   body           read-ply.ts:142-188 copies each row's properties into per-property
//                  TypedArrays.  Here: the element's rows stream file -> pinned chunk ->
//                  HBM (double-buffered, the pread of chunk k+1 overlapping the copy and
//                  transpose of chunk k) and k_ply_cols turns rows into columns:
//                  RB rows per workgroup staged in LDS with coalesced 4-byte loads, then
//                  one thread per (property, row) assembles the value's bytes and stores
//                  it (consecutive threads = consecutive rows of one column: coalesced).
//                  HBM traffic 2 x row bytes per row.
//   decompress     readers/decompress-ply.ts:82-232: one thread per splat, f64 JS
//                  semantics (lerp, unorm unpacking, Math.sqrt, V8's Math.log), f32
//                  stores; SH bytes -> floats.                   read 16 B + D, write 56 + 4D B
#include <fcntl.h>
#include <unistd.h>

#include <immintrin.h>
#include <sys/mman.h>

#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "st_internal.h"
#include "st_jsmath.h"

namespace st {
namespace {

// type_size: st_table.hip (st_internal.h)

int type_of(const std::string &s) {
    static const char *names[] = {"char", "uchar", "short", "ushort", "int", "uint", "float", "double"};
    for (int i = 0; i < 8; ++i)
        if (s == names[i]) return ST_PLY_CHAR + i;
    return 0;
}

// JS parseInt(s, 10); false for NaN
bool js_parse_int(const std::string &s, long long &v) {
    size_t i = 0;
    while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\r' || s[i] == '\v' || s[i] == '\f')) ++i;
    bool neg = false;
    if (i < s.size() && (s[i] == '+' || s[i] == '-')) neg = s[i++] == '-';
    size_t j = i;
    long long x = 0;
    while (j < s.size() && s[j] >= '0' && s[j] <= '9') {
        if (x < (1ll << 53)) x = x * 10 + (s[j] - '0');
        ++j;
    }
    if (j == i) return false;
    v = neg ? -x : x;
    return true;
}

void parse_header(const uint8_t *data, uint64_t len, st_ply_header *h) {
    std::memset(h, 0, sizeof *h);
    static const char magic[4] = {'p', 'l', 'y', '\n'};
    static const char end[12] = {'\n', 'e', 'n', 'd', '_', 'h', 'e', 'a', 'd', 'e', 'r', '\n'};
    ST_REQUIRE(len >= 16, ST_ERR_ARG, "ply: failed to read file header");
    ST_REQUIRE(std::memcmp(data, magic, 4) == 0, ST_ERR_ARG, "ply: invalid file header");
    // the reader grows the header byte by byte from 16 bytes until it ends with "\nend_header\n"
    uint64_t hs = 0;
    const uint64_t lim = len < 128 * 1024 ? len : 128 * 1024;
    for (uint64_t k = 17; k <= lim; ++k)
        if (std::memcmp(data + k - 12, end, 12) == 0) {
            hs = k;
            break;
        }
    ST_REQUIRE(hs, ST_ERR_ARG, "ply: failed to read file header");
    h->header_bytes = hs;
    // split on '\n', drop empty lines, skip the first line
    std::vector<std::string> lines;
    std::string cur;
    for (uint64_t i = 0; i < hs; ++i) {
        if (data[i] == '\n') {
            if (!cur.empty()) lines.push_back(cur);
            cur.clear();
        } else {
            cur.push_back((char)data[i]);
        }
    }
    if (!cur.empty()) lines.push_back(cur);
    st_ply_element *el = nullptr;
    std::string comments;
    for (size_t li = 1; li < lines.size(); ++li) {
        std::vector<std::string> w;
        size_t a = 0;
        const std::string &ln = lines[li];
        for (;;) {
            const size_t b = ln.find(' ', a);
            w.push_back(ln.substr(a, b == std::string::npos ? std::string::npos : b - a));
            if (b == std::string::npos) break;
            a = b + 1;
        }
        if (w[0] == "ply" || w[0] == "format" || w[0] == "end_header") continue;
        if (w[0] == "comment") {
            if (!comments.empty()) comments += '\n';
            comments += ln.size() > 8 ? ln.substr(8) : std::string();
            h->ncomments++;
        } else if (w[0] == "element") {
            ST_REQUIRE(w.size() == 3, ST_ERR_ARG, "ply: invalid ply header");
            ST_REQUIRE(h->nelements < ST_PLY_MAX_ELEMENTS, ST_ERR_UNSUPPORTED, "ply: too many elements");
            ST_REQUIRE(w[1].size() < ST_PLY_NAME, ST_ERR_UNSUPPORTED, "ply: element name too long");
            el = &h->elements[h->nelements++];
            std::memcpy(el->name, w[1].c_str(), w[1].size() + 1);
            long long cnt = 0;
            if (!js_parse_int(w[2], cnt)) cnt = 0;  // parseInt NaN: an empty element
            ST_REQUIRE(cnt >= 0, ST_ERR_ARG, "ply: invalid typed array length");
            el->count = (uint64_t)cnt;
        } else if (w[0] == "property") {
            ST_REQUIRE(el && w.size() == 3 && type_of(w[1]), ST_ERR_ARG, "ply: invalid ply header");
            ST_REQUIRE(el->nprops < ST_PLY_MAX_PROPS, ST_ERR_UNSUPPORTED, "ply: too many properties");
            ST_REQUIRE(w[2].size() < ST_PLY_NAME, ST_ERR_UNSUPPORTED, "ply: property name too long");
            st_ply_property &p = el->props[el->nprops++];
            std::memcpy(p.name, w[2].c_str(), w[2].size() + 1);
            p.type = type_of(w[1]);
        } else {
            throw Error(ST_ERR_ARG, "ply: unrecognized header value '" + w[0] + "' in ply header");
        }
    }
    ST_REQUIRE(comments.size() < sizeof h->comments, ST_ERR_UNSUPPORTED, "ply: comments too long");
    std::memcpy(h->comments, comments.c_str(), comments.size() + 1);
}

uint32_t row_bytes(const st_ply_element &e) {
    uint32_t r = 0;
    for (int p = 0; p < e.nprops; ++p) r += type_size(e.props[p].type);
    return r;
}

struct PropSlot {
    uint32_t offset;  // byte offset in the row
    uint32_t size;    // 1, 2, 4, 8
};

constexpr uint32_t LDS_ROWS_BYTES = 48 * 1024;
// pread threads per file chunk (ST_PLY_READERS: tuning experiments)
const int kReaders = std::max(1, std::min(32, std::getenv("ST_PLY_READERS") ? std::atoi(std::getenv("ST_PLY_READERS")) : 8));

// rows [0, nrows) of the staged chunk -> columns at rows [row0, row0 + nrows)
__global__ __launch_bounds__(256) void k_ply_cols(const uint8_t *__restrict__ rows, uint64_t nrows, uint32_t R,
                                                  uint32_t RB, const PropSlot *__restrict__ props, int nprops,
                                                  void *const *__restrict__ cols, uint64_t row0) {
    extern __shared__ uint32_t lds32[];
    const uint8_t *lds8 = (const uint8_t *)lds32;
    const uint64_t r0 = (uint64_t)blockIdx.x * RB;
    const uint32_t nr = (uint32_t)((nrows - r0) < RB ? (nrows - r0) : RB);
    // RB is a multiple of 4, so every block starts 4-byte aligned; a partial last word is
    // read byte by byte (never past the rows)
    const uint32_t bytes = nr * R, words = bytes / 4;
    const uint32_t *src = (const uint32_t *)(rows + r0 * R);
    for (uint32_t i = threadIdx.x; i < words; i += 256) lds32[i] = src[i];
    if (threadIdx.x == 0 && (bytes & 3)) {
        uint32_t v = 0;
        for (uint32_t k = 0; k < (bytes & 3); ++k) v |= (uint32_t)rows[r0 * R + words * 4 + k] << (8 * k);
        lds32[words] = v;
    }
    __syncthreads();
    const uint32_t total = nr * (uint32_t)nprops;
    for (uint32_t e = threadIdx.x; e < total; e += 256) {
        const uint32_t p = e / nr, r = e - p * nr;
        const PropSlot ps = props[p];
        const uint32_t off = r * R + ps.offset;
        uint64_t v = 0;
        for (uint32_t k = 0; k < ps.size; ++k) v |= (uint64_t)lds8[off + k] << (8 * k);
        const uint64_t row = row0 + r0 + r;
        switch (ps.size) {
            case 1: ((uint8_t *)cols[p])[row] = (uint8_t)v; break;
            case 2: ((uint16_t *)cols[p])[row] = (uint16_t)v; break;
            case 4: ((uint32_t *)cols[p])[row] = (uint32_t)v; break;
            default: ((uint64_t *)cols[p])[row] = v; break;
        }
    }
}

struct Transposer {
    st_ctx *c;
    uint32_t R, RB;
    int nprops;
    PropSlot *d_props;
    void **d_cols;
    Transposer(st_ctx *ctx, const st_ply_element &e, void *const *cols, const std::string &tag) : c(ctx) {
        R = row_bytes(e);
        nprops = e.nprops;
        RB = R ? (LDS_ROWS_BYTES / R) & ~3u : 64;
        ST_REQUIRE(R == 0 || RB >= 4, ST_ERR_UNSUPPORTED, "ply: rows longer than 12 KiB");
        if (RB > 256) RB = 256;
        std::vector<PropSlot> ps(nprops);
        uint32_t off = 0;
        for (int p = 0; p < nprops; ++p) {
            ps[p] = {off, (uint32_t)type_size(e.props[p].type)};
            off += ps[p].size;
        }
        d_props = wsT<PropSlot>(c, tag + ".props", nprops ? nprops : 1);
        d_cols = wsT<void *>(c, tag + ".cols", nprops ? nprops : 1);
        if (nprops) {
            ST_HIP(hipMemcpyAsync(d_props, ps.data(), sizeof(PropSlot) * nprops, hipMemcpyHostToDevice, c->stream));
            ST_HIP(hipMemcpyAsync(d_cols, cols, sizeof(void *) * nprops, hipMemcpyHostToDevice, c->stream));
        }
    }
    void run(const uint8_t *rows, uint64_t nrows, uint64_t row0) {
        if (!nrows || !nprops) return;
        KTimer kt(c, "ply.cols");
        hipLaunchKernelGGL(k_ply_cols, dim3((unsigned)((nrows + RB - 1) / RB)), dim3(256), (RB * R + 3) & ~3u,
                           c->stream, rows, nrows, R, RB, d_props, nprops, (void *const *)d_cols, row0);
        ST_LAUNCH_CHECK();
    }
};

// ---- compressed PLY -------------------------------------------------------------
struct DecompArgs {
    const float *chunk[18];
    const uint32_t *vertex[4];
    float *out[14];
};

__device__ inline double unorm(uint32_t v, int bits) {
    const uint32_t t = (1u << bits) - 1;
    return (double)(v & t) / (double)t;
}
__device__ inline double lerp(double a, double b, double t) { return a * (1 - t) + b * t; }

__global__ __launch_bounds__(256) void k_decompress(DecompArgs A, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint64_t ci = i / 256;
    const uint32_t pp = A.vertex[0][i], pr = A.vertex[1][i], ps = A.vertex[2][i], pc = A.vertex[3][i];
    const double px = unorm(pp >> 21, 11), py = unorm(pp >> 11, 10), pz = unorm(pp, 11);
    const double sx = unorm(ps >> 21, 11), sy = unorm(ps >> 11, 10), sz = unorm(ps, 11);
    const double cx = unorm(pc >> 24, 8), cy = unorm(pc >> 16, 8), cz = unorm(pc >> 8, 8), cw = unorm(pc, 8);
    const double norm = 1.0 / (__builtin_sqrt(2.0) * 0.5);
    const double a = (unorm(pr >> 20, 10) - 0.5) * norm;
    const double b = (unorm(pr >> 10, 10) - 0.5) * norm;
    const double c = (unorm(pr, 10) - 0.5) * norm;
    const double s2 = 1.0 - (a * a + b * b + c * c);
    const double m = __builtin_sqrt(s2 > 0 ? s2 : 0.0);  // Math.max(0, x) of a finite x
    const uint32_t which = pr >> 30;
    const double r0 = which == 0 ? m : a;
    const double r1 = which == 0 ? a : (which == 1 ? m : b);
    const double r2 = which <= 1 ? b : (which == 2 ? m : c);
    const double r3 = which <= 2 ? c : m;
    A.out[0][i] = (float)lerp(A.chunk[0][ci], A.chunk[3][ci], px);
    A.out[1][i] = (float)lerp(A.chunk[1][ci], A.chunk[4][ci], py);
    A.out[2][i] = (float)lerp(A.chunk[2][ci], A.chunk[5][ci], pz);
    const double SH_C0 = 0.28209479177387814;
    A.out[3][i] = (float)((lerp(A.chunk[12][ci], A.chunk[15][ci], cx) - 0.5) / SH_C0);
    A.out[4][i] = (float)((lerp(A.chunk[13][ci], A.chunk[16][ci], cy) - 0.5) / SH_C0);
    A.out[5][i] = (float)((lerp(A.chunk[14][ci], A.chunk[17][ci], cz) - 0.5) / SH_C0);
    A.out[6][i] = (float)(-js::log(1 / cw - 1));
    A.out[7][i] = (float)r0;
    A.out[8][i] = (float)r1;
    A.out[9][i] = (float)r2;
    A.out[10][i] = (float)r3;
    A.out[11][i] = (float)lerp(A.chunk[6][ci], A.chunk[9][ci], sx);
    A.out[12][i] = (float)lerp(A.chunk[7][ci], A.chunk[10][ci], sy);
    A.out[13][i] = (float)lerp(A.chunk[8][ci], A.chunk[11][ci], sz);
}

constexpr int SH_MAX = 45;
struct ShArgs {
    const uint8_t *sh[SH_MAX];
    float *out[SH_MAX];
};

__global__ __launch_bounds__(256) void k_decompress_sh(ShArgs A, int nsh, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    for (int k = 0; k < nsh; ++k) {
        const uint32_t v = A.sh[k][i];
        const double t = (v == 0) ? 0.0 : (v == 255) ? 1.0 : (v + 0.5) / 256;
        A.out[k][i] = (float)((t - 0.5) * 8);
    }
}

}  // namespace

void decompress_ply_dev(st_ctx *c, uint64_t n, const float *const *chunk, const uint32_t *const *vertex,
                        const uint8_t *const *sh, int nsh, float *const *out) {
    ST_REQUIRE(nsh == 0 || nsh == 9 || nsh == 24 || nsh == 45, ST_ERR_ARG,
               "decompress: SH column count must be 0, 9, 24 or 45 (decompress-ply.ts:62)");
    if (!n) return;
    DecompArgs A{};
    for (int k = 0; k < 18; ++k) A.chunk[k] = chunk[k];
    for (int k = 0; k < 4; ++k) A.vertex[k] = vertex[k];
    for (int k = 0; k < 14; ++k) A.out[k] = out[k];
    {
        KTimer kt(c, "ply.decompress");
        hipLaunchKernelGGL(k_decompress, dim3(grid_for(n, 256)), dim3(256), 0, c->stream, A, n);
        ST_LAUNCH_CHECK();
    }
    if (nsh) {
        ShArgs S{};
        for (int k = 0; k < nsh; ++k) {
            S.sh[k] = sh[k];
            S.out[k] = out[14 + k];
        }
        hipLaunchKernelGGL(k_decompress_sh, dim3(grid_for(n, 256)), dim3(256), 0, c->stream, S, nsh, n);
        ST_LAUNCH_CHECK();
    }
}

// one element of a PLY file (fd) into device columns, streamed through pinned chunks; a sink
// (st_ply_read) also gets every chunk on the host
void ply_read_dev(st_ctx *c, int fd, const st_ply_header &h, int element, void *const *cols, ChunkSink *sink) {
    ST_REQUIRE(element >= 0 && element < h.nelements, ST_ERR_ARG, "ply: element index out of range");
    uint64_t off = h.header_bytes;
    for (int e = 0; e < element; ++e) off += h.elements[e].count * row_bytes(h.elements[e]);
    const st_ply_element &el = h.elements[element];
    Transposer tp(c, el, cols, "ply");
    const uint64_t R = tp.R, total = el.count * R;
    if (!total) return;
    // chunks of whole LDS blocks, ~64 MiB (ST_PLY_CHUNK overrides the byte target: tests)
    uint64_t target = 64ull << 20;
    if (const char *e = std::getenv("ST_PLY_CHUNK")) target = std::strtoull(e, nullptr, 10);
    const uint64_t per = (uint64_t)tp.RB * R;
    const uint64_t chunk_rows = (target / per > 0 ? target / per : 1) * tp.RB;
    const uint64_t chunk_bytes = chunk_rows * R;
    uint8_t *pin = (uint8_t *)io_buf(c, 2 * (chunk_bytes + 64));
    uint8_t *stage[2] = {wsT<uint8_t>(c, "ply.stage0", chunk_bytes + 64), wsT<uint8_t>(c, "ply.stage1", chunk_bytes + 64)};
    hipEvent_t ev[2];
    ST_HIP(hipEventCreateWithFlags(&ev[0], hipEventDisableTiming));
    ST_HIP(hipEventCreateWithFlags(&ev[1], hipEventDisableTiming));
    bool pending[2] = {false, false};
    try {
        uint64_t row = 0;
        for (int k = 0; row < el.count; ++k) {
            const int b = k & 1;
            const uint64_t nr = (el.count - row) < chunk_rows ? (el.count - row) : chunk_rows;
            const uint64_t bytes = nr * R;
            uint8_t *hb = pin + b * (chunk_bytes + 64);
            if (pending[b]) ST_HIP(hipEventSynchronize(ev[b]));  // the copy out of hb is done
            if (sink) sink->wait(b);                              // and the host's pass over it
            // page-cache copies are per-thread memcpy bound: several readers per chunk
            const uint64_t base = off + row * R;
            const int nt = bytes >= (8ull << 20) ? kReaders : 1;
            std::vector<std::thread> th;
            std::vector<int> ok(nt, 1);
            for (int t = 0; t < nt; ++t) {
                const uint64_t a0 = bytes * t / nt, a1 = bytes * (t + 1) / nt;
                auto job = [&, t, a0, a1] {
                    uint64_t got = a0;
                    while (got < a1) {
                        const ssize_t r = pread(fd, hb + got, a1 - got, (off_t)(base + got));
                        if (r <= 0) {
                            ok[t] = 0;
                            return;
                        }
                        got += (uint64_t)r;
                    }
                };
                if (nt == 1)
                    job();
                else
                    th.emplace_back(job);
            }
            for (auto &x : th) x.join();
            for (int t = 0; t < nt; ++t)
                ST_REQUIRE(ok[t], ST_ERR_ARG, "ply: file shorter than its header declares");
            ST_HIP(hipMemcpyAsync(stage[b], hb, bytes, hipMemcpyHostToDevice, c->stream));
            ST_HIP(hipEventRecord(ev[b], c->stream));
            pending[b] = true;
            tp.run(stage[b], nr, row);
            if (sink) sink->take(b, hb, row, nr);
            row += nr;
        }
        ST_HIP(hipStreamSynchronize(c->stream));
    } catch (...) {
        (void)hipStreamSynchronize(c->stream);
        (void)hipEventDestroy(ev[0]);
        (void)hipEventDestroy(ev[1]);
        throw;
    }
    (void)hipEventDestroy(ev[0]);
    (void)hipEventDestroy(ev[1]);
}

// ---- st_ply_read: the host columns transposed on the host ------------------------------------
// The rows of every pinned chunk go up to HBM and are transposed there (ply_read_dev: the device
// columns, kept as the mirrors of st_ctx::HostMirror), and the same pinned rows are transposed
// into the caller's host columns by the host's copy threads while the next chunk is read -- the
// columns never cross the link back.  A float-only element (every 3DGS PLY) moves in 8 x 8
// blocks of AVX2 registers; other property types one value at a time.  The host transpose also
// writes the columns' pristine twin (c->shadow) that the writeSog host forms compare against.
namespace {

struct Props {
    std::vector<uint32_t> off, sz;  // byte offset in the row, size
    uint32_t R = 0;
    bool all4 = true;
};

// rows [i0, i1) of the chunk (row r of the element at chunk row r - row0) into dst (+ dst2)
void transpose_scalar(const uint8_t *rows, uint64_t row0, uint64_t i0, uint64_t i1, const Props &P,
                      void *const *dst, void *const *dst2) {
    const int np = (int)P.sz.size();
    for (uint64_t i = i0; i < i1; ++i) {
        const uint8_t *src = rows + i * P.R;
        const uint64_t r = row0 + i;
        for (int p = 0; p < np; ++p) {
            const uint32_t z = P.sz[p];
            for (int k = 0; k < 2; ++k) {
                void *d = k ? (dst2 ? dst2[p] : nullptr) : dst[p];
                if (!d) continue;
                std::memcpy(static_cast<uint8_t *>(d) + r * z, src + P.off[p], z);
            }
        }
    }
}

// 8 rows x 8 float columns (row stride `stride` floats) -> c[k] = column k of the 8 rows
__attribute__((target("avx2"))) inline void t8x8(const float *s0, uint64_t stride, __m256 c[8]) {
    const __m256 r0 = _mm256_loadu_ps(s0), r1 = _mm256_loadu_ps(s0 + stride), r2 = _mm256_loadu_ps(s0 + 2 * stride),
                 r3 = _mm256_loadu_ps(s0 + 3 * stride), r4 = _mm256_loadu_ps(s0 + 4 * stride),
                 r5 = _mm256_loadu_ps(s0 + 5 * stride), r6 = _mm256_loadu_ps(s0 + 6 * stride),
                 r7 = _mm256_loadu_ps(s0 + 7 * stride);
    const __m256 t0 = _mm256_unpacklo_ps(r0, r1), t1 = _mm256_unpackhi_ps(r0, r1);
    const __m256 t2 = _mm256_unpacklo_ps(r2, r3), t3 = _mm256_unpackhi_ps(r2, r3);
    const __m256 t4 = _mm256_unpacklo_ps(r4, r5), t5 = _mm256_unpackhi_ps(r4, r5);
    const __m256 t6 = _mm256_unpacklo_ps(r6, r7), t7 = _mm256_unpackhi_ps(r6, r7);
    const __m256 u0 = _mm256_shuffle_ps(t0, t2, 0x44), u1 = _mm256_shuffle_ps(t0, t2, 0xEE);
    const __m256 u2 = _mm256_shuffle_ps(t1, t3, 0x44), u3 = _mm256_shuffle_ps(t1, t3, 0xEE);
    const __m256 u4 = _mm256_shuffle_ps(t4, t6, 0x44), u5 = _mm256_shuffle_ps(t4, t6, 0xEE);
    const __m256 u6 = _mm256_shuffle_ps(t5, t7, 0x44), u7 = _mm256_shuffle_ps(t5, t7, 0xEE);
    c[0] = _mm256_permute2f128_ps(u0, u4, 0x20);
    c[1] = _mm256_permute2f128_ps(u1, u5, 0x20);
    c[2] = _mm256_permute2f128_ps(u2, u6, 0x20);
    c[3] = _mm256_permute2f128_ps(u3, u7, 0x20);
    c[4] = _mm256_permute2f128_ps(u0, u4, 0x31);
    c[5] = _mm256_permute2f128_ps(u1, u5, 0x31);
    c[6] = _mm256_permute2f128_ps(u2, u6, 0x31);
    c[7] = _mm256_permute2f128_ps(u3, u7, 0x31);
}

// Every column 64-B aligned (the addon's column blocks, the host twins): 16 rows at a time, each
// column's 64 bytes of them one whole cache line written with two streaming stores -- no read
// for ownership of the 2.5 GB of columns, no cache pollution.  Otherwise 8 rows at a time with
// ordinary stores.  The last np % 8 columns and the rows outside whole groups go value by value.
__attribute__((target("avx2"))) void transpose_f32_avx2(const uint8_t *rows, uint64_t row0, uint64_t i0, uint64_t i1,
                                                        const Props &P, void *const *dst, void *const *dst2) {
    const int np = (int)P.sz.size(), nb = np / 8;
    const uint64_t stride = P.R / 4;
    bool aligned = true;
    for (int p = 0; p < np; ++p) {
        aligned = aligned && ((uintptr_t)dst[p] & 63) == 0;
        if (dst2) aligned = aligned && ((uintptr_t)dst2[p] & 63) == 0;
    }
    uint64_t i = i0;
    __m256 c[8], e[8];
    if (aligned) {
        const uint64_t head = std::min(i1, i0 + ((16 - ((row0 + i0) & 15)) & 15));  // to a 16-row boundary
        transpose_scalar(rows, row0, i0, head, P, dst, dst2);
        for (i = head; i + 16 <= i1; i += 16) {
            const float *src = reinterpret_cast<const float *>(rows + i * P.R);
            const uint64_t r = row0 + i;
            for (int j = 0; j < nb; ++j) {
                t8x8(src + 8 * j, stride, c);
                t8x8(src + 8 * stride + 8 * j, stride, e);
                for (int k = 0; k < 8; ++k) {
                    float *d = static_cast<float *>(dst[8 * j + k]) + r;
                    _mm256_stream_ps(d, c[k]);
                    _mm256_stream_ps(d + 8, e[k]);
                    if (dst2) {
                        float *d2 = static_cast<float *>(dst2[8 * j + k]) + r;
                        _mm256_stream_ps(d2, c[k]);
                        _mm256_stream_ps(d2 + 8, e[k]);
                    }
                }
            }
            for (int p = 8 * nb; p < np; ++p)  // the last np % 8 columns
                for (int k = 0; k < 16; ++k) {
                    const float v = src[k * stride + p];
                    static_cast<float *>(dst[p])[r + k] = v;
                    if (dst2) static_cast<float *>(dst2[p])[r + k] = v;
                }
        }
        _mm_sfence();  // the streaming stores are visible before the copy thread reports done
    } else {
        for (; i + 8 <= i1; i += 8) {
            const float *src = reinterpret_cast<const float *>(rows + i * P.R);
            const uint64_t r = row0 + i;
            for (int j = 0; j < nb; ++j) {
                t8x8(src + 8 * j, stride, c);
                for (int k = 0; k < 8; ++k) {
                    _mm256_storeu_ps(static_cast<float *>(dst[8 * j + k]) + r, c[k]);
                    if (dst2) _mm256_storeu_ps(static_cast<float *>(dst2[8 * j + k]) + r, c[k]);
                }
            }
            for (int p = 8 * nb; p < np; ++p)
                for (int k = 0; k < 8; ++k) {
                    const float v = src[k * stride + p];
                    static_cast<float *>(dst[p])[r + k] = v;
                    if (dst2) static_cast<float *>(dst2[p])[r + k] = v;
                }
        }
    }
    transpose_scalar(rows, row0, i, i1, P, dst, dst2);
}

bool has_avx2() {
    static const bool yes = __builtin_cpu_supports("avx2");
    return yes;
}

// the copy threads transpose each chunk while the reader fills the other buffer
struct HostTranspose : ChunkSink {
    st_ctx *c;
    const Props &P;
    void *const *dst;
    void *const *dst2;
    std::mutex mu;
    std::condition_variable cv;
    struct Job {
        int b;
        const uint8_t *rows;
        uint64_t row, nr;
    };
    std::deque<Job> q;
    bool busy[2] = {false, false}, fin = false;
    std::exception_ptr err;
    std::thread th;
    HostTranspose(st_ctx *ctx, const Props &p, void *const *d, void *const *d2) : c(ctx), P(p), dst(d), dst2(d2) {
        th = std::thread([this] { loop(); });
    }
    void loop() {
        for (;;) {
            Job j;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return fin || !q.empty(); });
                if (q.empty()) return;
                j = q.front();
                q.pop_front();
            }
            try {
                const bool vec = P.all4 && P.R == 4 * P.sz.size() && has_avx2();
                host_parallel(c, [&](int t, int nt) {
                    // 16-row shares (the AVX2 blocks' cache lines), the remainder to the last thread
                    const uint64_t blocks = j.nr / 16, a = blocks * t / nt * 16,
                                   e = (t == nt - 1) ? j.nr : blocks * (t + 1) / nt * 16;
                    if (vec) transpose_f32_avx2(j.rows, j.row, a, e, P, dst, dst2);
                    else transpose_scalar(j.rows, j.row, a, e, P, dst, dst2);
                });
            } catch (...) {
                std::lock_guard<std::mutex> lk(mu);
                if (!err) err = std::current_exception();
            }
            {
                std::lock_guard<std::mutex> lk(mu);
                busy[j.b] = false;
            }
            cv.notify_all();
        }
    }
    void take(int b, const uint8_t *rows, uint64_t row, uint64_t nr) override {
        {
            std::lock_guard<std::mutex> lk(mu);
            busy[b] = true;
            q.push_back({b, rows, row, nr});
        }
        cv.notify_all();
    }
    void wait(int b) override {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return !busy[b]; });
    }
    void finish() {
        {
            std::lock_guard<std::mutex> lk(mu);
            fin = true;
        }
        cv.notify_all();
        if (th.joinable()) th.join();
    }
    ~HostTranspose() override { finish(); }
};

}  // namespace

// the mirrors `pick` selects dropped, the lazy ones among them first copied down into their host
// columns
void materialize_where(st_ctx *c, const std::function<bool(const st_ctx::HostMirror &)> &pick) {
    std::vector<HostXfer> xs;
    std::lock_guard<std::mutex> lk(c->mirror_mu);
    if (c->mirrors.empty()) return;
    for (const auto &m : c->mirrors)
        if (pick(m) && m.lazy && m.bytes)
            xs.push_back(HostXfer{const_cast<void *>(m.host), const_cast<void *>(m.dev), (size_t)m.bytes});
    if (!xs.empty()) staged_d2h_raw(c, xs);
    drop_mirrors_locked(c, pick);
}

// (mirror_mu held) the mirrors `pick` selects removed; their own device blocks go to the pool
void drop_mirrors_locked(st_ctx *c, const std::function<bool(const st_ctx::HostMirror &)> &pick) {
    std::vector<st_ctx::HostMirror> keep;
    for (const auto &m : c->mirrors) {
        if (!pick(m)) {
            keep.push_back(m);
            continue;
        }
        if (m.dev_bytes) c->dev_pool.emplace_back(const_cast<void *>(m.dev), m.dev_bytes);
    }
    c->mirrors.swap(keep);
}

// (mirror_mu held) a device block of `bytes` for a resident column: a pooled one of that size, or
// a new one (the pool is trimmed to ST_PLY_POOL_MB, default 16384, first)
void *resident_block_locked(st_ctx *c, uint64_t bytes) {
    for (size_t i = c->dev_pool.size(); i-- > 0;)
        if (c->dev_pool[i].second == bytes) {
            void *p = c->dev_pool[i].first;
            c->dev_pool.erase(c->dev_pool.begin() + (long)i);
            return p;
        }
    static const uint64_t cap = (uint64_t)(getenv("ST_PLY_POOL_MB") ? atoll(getenv("ST_PLY_POOL_MB")) : 16384) << 20;
    uint64_t held = 0;
    for (auto &b : c->dev_pool) held += b.second;
    while (!c->dev_pool.empty() && held + bytes > cap) {
        held -= c->dev_pool.front().second;
        ST_HIP(hipFree(c->dev_pool.front().first));
        c->dev_pool.erase(c->dev_pool.begin());
    }
    void *p = nullptr;
    ST_HIP(hipMalloc(&p, bytes));
    return p;
}

bool overlaps(const st_ctx::HostMirror &m, const void *p, size_t bytes) {
    const char *a = static_cast<const char *>(m.host), *b = static_cast<const char *>(p);
    return bytes && m.bytes && b < a + m.bytes && a < b + bytes;
}

void materialize_lazy(st_ctx *c, const void *const *host, int n) {
    materialize_where(c, [&](const st_ctx::HostMirror &m) {
        if (!m.lazy) return false;
        for (int i = 0; i < n; ++i)
            if (host[i] == m.host) return true;
        return false;
    });
}

// staged_h2d's sources: a lazy column about to be read from host memory is copied down first
void mirrors_before_h2d(st_ctx *c, const std::vector<HostXfer> &xs) {
    materialize_where(c, [&](const st_ctx::HostMirror &m) {
        if (!m.lazy) return false;
        for (const auto &x : xs)
            if (overlaps(m, x.host, x.bytes)) return true;
        return false;
    });
}

// staged_d2h's destinations: a host column about to be overwritten is no longer its device copy's
// mirror (lazy or not: dropped without copying)
void mirrors_before_d2h(st_ctx *c, const std::vector<HostXfer> &xs) {
    std::lock_guard<std::mutex> lk(c->mirror_mu);
    if (c->mirrors.empty()) return;
    drop_mirrors_locked(c, [&](const st_ctx::HostMirror &m) {
        for (const auto &x : xs)
            if (overlaps(m, x.host, x.bytes)) return true;
        return false;
    });
}

void ply_read_host(st_ctx *c, int fd, const st_ply_header &h, int element, void *const *host_cols, bool lazy) {
    const st_ply_element &el = h.elements[element];
    const int np = el.nprops;
    Props P;
    std::vector<void *> dcols(np), twins(np);
    std::vector<uint64_t> toff(np), dbytes(np);
    uint64_t total = 0;
    for (int p = 0; p < np; ++p) {
        const uint32_t z = (uint32_t)type_size(el.props[p].type);
        P.off.push_back(P.R);
        P.sz.push_back(z);
        P.R += z;
        P.all4 = P.all4 && z == 4;
        dbytes[p] = el.count * z + 8;
        toff[p] = total;
        total += (el.count * z + 63) / 64 * 64;
    }
    if (lazy) {
        // the rows go up and are transposed in HBM only, into blocks of the columns' own (no other
        // read reuses them); the host columns stay unfilled until st_ply_materialize (or a host form
        // other than writeSog's) asks for them
        {
            std::lock_guard<std::mutex> lk(c->mirror_mu);
            for (int p = 0; p < np; ++p) dcols[p] = el.count ? resident_block_locked(c, dbytes[p]) : nullptr;
        }
        using clk = std::chrono::steady_clock;
        const auto t0 = clk::now();
        try {
            if (el.count) ply_read_dev(c, fd, h, element, dcols.data(), nullptr);
            ST_HIP(hipStreamSynchronize(c->stream));
        } catch (...) {
            std::lock_guard<std::mutex> lk(c->mirror_mu);
            for (int p = 0; p < np; ++p)
                if (dcols[p]) c->dev_pool.emplace_back(dcols[p], dbytes[p]);
            throw;
        }
        if (std::getenv("ST_DEBUG"))
            fprintf(stderr, "[st ply read] %.1f MB: device columns %.1f ms (host columns resident)\n", total / 1e6,
                    std::chrono::duration<double, std::milli>(clk::now() - t0).count());
        std::lock_guard<std::mutex> lk(c->mirror_mu);
        // a host column registered before at the same address (its memory reused) is not that one
        drop_mirrors_locked(c, [&](const st_ctx::HostMirror &m) {
            for (int p = 0; p < np; ++p)
                if (m.host == host_cols[p]) return true;
            return false;
        });
        if (el.count)  // (an empty element has nothing to keep)
            for (int p = 0; p < np; ++p)
                c->mirrors.push_back({host_cols[p], el.count * P.sz[p], nullptr, dcols[p], element, true, dbytes[p]});
        return;
    }
    // an eager read overwrites this element's device slots and the shared host twins: every other
    // eager mirror goes (the resident ones keep blocks of their own)
    {
        std::lock_guard<std::mutex> lk(c->mirror_mu);
        drop_mirrors_locked(c, [&](const st_ctx::HostMirror &m) {
            if (!m.lazy) return true;
            for (int p = 0; p < np; ++p)
                if (m.host == host_cols[p]) return true;
            return false;
        });
    }
    for (int p = 0; p < np; ++p)
        dcols[p] = ws(c, "plyh.e" + std::to_string(element) + ".c" + std::to_string(p), dbytes[p]);
    const char *mo = std::getenv("ST_HOST_MIRROR");
    const bool mirror = !(mo && std::strcmp(mo, "0") == 0) && el.count && np;
    if (mirror && c->shadow_bytes < total) {
        std::free(c->shadow);
        c->shadow = nullptr;
        c->shadow_bytes = 0;
        const size_t huge = 2u << 20, len = (total + huge - 1) / huge * huge;
        ST_REQUIRE(posix_memalign(&c->shadow, huge, len) == 0, ST_ERR_NOMEM, "ply: host twin allocation failed");
        madvise(c->shadow, len, MADV_HUGEPAGE);
        c->shadow_bytes = len;
    }
    for (int p = 0; p < np; ++p) twins[p] = mirror ? static_cast<uint8_t *>(c->shadow) + toff[p] : nullptr;
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    {
        HostTranspose sink(c, P, host_cols, mirror ? twins.data() : nullptr);
        ply_read_dev(c, fd, h, element, dcols.data(), el.count ? &sink : nullptr);
        sink.finish();
        if (sink.err) std::rethrow_exception(sink.err);
    }
    if (std::getenv("ST_DEBUG"))
        fprintf(stderr, "[st ply read] %.1f MB: device and host columns %.1f ms (%s host transpose)\n", total / 1e6,
                std::chrono::duration<double, std::milli>(clk::now() - t0).count(),
                P.all4 && P.R == 4 * (uint32_t)np && has_avx2() ? "AVX2" : "scalar");
    if (mirror) {
        std::lock_guard<std::mutex> lk(c->mirror_mu);
        for (int p = 0; p < np; ++p)
            c->mirrors.push_back({host_cols[p], el.count * P.sz[p], twins[p], dcols[p], element, false});
    }
}

}  // namespace st

using namespace st;

extern "C" {

int st_ply_parse_header(const uint8_t *data, uint64_t len, st_ply_header *out) {
    return guard([&] {
        ST_REQUIRE(data && out, ST_ERR_ARG, "NULL argument");
        parse_header(data, len, out);
    });
}

int st_ply_read_header(int32_t fd, st_ply_header *out) {
    return guard([&] {
        ST_REQUIRE(out && fd >= 0, ST_ERR_ARG, "bad argument");
        std::vector<uint8_t> buf(128 * 1024);
        uint64_t got = 0;
        for (;;) {
            const ssize_t r = pread(fd, buf.data() + got, buf.size() - got, (off_t)got);
            if (r <= 0) break;
            got += (uint64_t)r;
            if (got == buf.size()) break;
        }
        parse_header(buf.data(), got, out);
    });
}

uint64_t st_ply_row_bytes(const st_ply_header *h, int32_t element) {
    if (!h || element < 0 || element >= h->nelements) return 0;
    return row_bytes(h->elements[element]);
}

int st_dev_ply_transpose(st_ctx *c, const st_ply_header *h, int32_t element, const uint8_t *rows, uint64_t nrows,
                         void *const *cols) {
    return guard([&] {
        ST_REQUIRE(c && h && rows && cols && element >= 0 && element < h->nelements, ST_ERR_ARG, "bad argument");
        ST_REQUIRE(((uintptr_t)rows & 3) == 0, ST_ERR_ARG, "ply: rows must be 4-byte aligned");
        use_device(c);
        Transposer tp(c, h->elements[element], cols, "plyt");
        tp.run(rows, nrows, 0);
    });
}

int st_dev_ply_read(st_ctx *c, int32_t fd, const st_ply_header *h, int32_t element, void *const *cols) {
    return guard([&] {
        ST_REQUIRE(c && h && cols && fd >= 0, ST_ERR_ARG, "bad argument");
        use_device(c);
        ply_read_dev(c, fd, *h, element, cols);
    });
}

int st_ply_read(st_ctx *c, int32_t fd, const st_ply_header *h, int32_t element, void *const *host_cols) {
    return guard([&] {
        ST_REQUIRE(c && h && host_cols && fd >= 0 && element >= 0 && element < h->nelements, ST_ERR_ARG,
                   "bad argument");
        use_device(c);
        ply_read_host(c, fd, *h, element, host_cols);
    });
}

int st_ply_read_resident(st_ctx *c, int32_t fd, const st_ply_header *h, int32_t element, void *const *host_cols) {
    return guard([&] {
        ST_REQUIRE(c && h && host_cols && fd >= 0 && element >= 0 && element < h->nelements, ST_ERR_ARG,
                   "bad argument");
        for (int32_t p = 0; p < h->elements[element].nprops; ++p)
            ST_REQUIRE(host_cols[p] || !h->elements[element].count, ST_ERR_ARG, "ply: NULL host column");
        use_device(c);
        ply_read_host(c, fd, *h, element, host_cols, true);
    });
}

int st_ply_materialize(st_ctx *c, const void *host_col) {
    return guard([&] {
        ST_REQUIRE(c, ST_ERR_ARG, "NULL context");
        use_device(c);
        if (host_col) materialize_lazy(c, &host_col, 1);
    });
}

int st_ply_forget(st_ctx *c, const void *host_col) {
    return guard([&] {
        ST_REQUIRE(c, ST_ERR_ARG, "NULL context");
        std::lock_guard<std::mutex> lk(c->mirror_mu);
        drop_mirrors_locked(c, [&](const st_ctx::HostMirror &m) { return m.host == host_col; });
    });
}

int st_dev_decompress_ply(st_ctx *c, uint64_t n, const float *const *chunk, const uint32_t *const *vertex,
                          const uint8_t *const *sh, int32_t nsh, float *const *out) {
    return guard([&] {
        ST_REQUIRE(c && chunk && vertex && out && (nsh == 0 || sh), ST_ERR_ARG, "NULL argument");
        use_device(c);
        decompress_ply_dev(c, n, chunk, vertex, sh, nsh, out);
    });
}

int st_decompress_ply(st_ctx *c, uint64_t n, const float *const *chunk, const uint32_t *const *vertex,
                      const uint8_t *const *sh, int32_t nsh, float *const *out) {
    return guard([&] {
        ST_REQUIRE(c && chunk && vertex && out && (nsh == 0 || sh), ST_ERR_ARG, "NULL argument");
        ST_REQUIRE(nsh == 0 || nsh == 9 || nsh == 24 || nsh == 45, ST_ERR_ARG,
                   "decompress: SH column count must be 0, 9, 24 or 45 (decompress-ply.ts:62)");
        use_device(c);
        const uint64_t nch = (n + 255) / 256;
        std::vector<const float *> dchunk(18);
        std::vector<const uint32_t *> dvert(4);
        std::vector<const uint8_t *> dsh(nsh);
        std::vector<float *> dout(14 + nsh);
        std::vector<HostXfer> up;
        for (int k = 0; k < 18; ++k) {
            float *d = wsT<float>(c, "dph.ch" + std::to_string(k), nch);
            up.push_back(HostXfer{const_cast<float *>(chunk[k]), d, nch * 4});
            dchunk[k] = d;
        }
        for (int k = 0; k < 4; ++k) {
            uint32_t *d = wsT<uint32_t>(c, "dph.v" + std::to_string(k), n);
            up.push_back(HostXfer{const_cast<uint32_t *>(vertex[k]), d, n * 4});
            dvert[k] = d;
        }
        for (int k = 0; k < nsh; ++k) {
            uint8_t *d = wsT<uint8_t>(c, "dph.s" + std::to_string(k), n);
            up.push_back(HostXfer{const_cast<uint8_t *>(sh[k]), d, n});
            dsh[k] = d;
        }
        staged_h2d(c, up);
        for (int k = 0; k < 14 + nsh; ++k) dout[k] = wsT<float>(c, "dph.o" + std::to_string(k), n);
        decompress_ply_dev(c, n, dchunk.data(), dvert.data(), dsh.data(), nsh, dout.data());
        std::vector<HostXfer> down;
        for (int k = 0; k < 14 + nsh; ++k) down.push_back(HostXfer{out[k], dout[k], n * 4});
        staged_d2h(c, down);
    });
}

}  // extern "C"
