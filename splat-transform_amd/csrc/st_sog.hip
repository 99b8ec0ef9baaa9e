// st_sog.hip -- writeSog texture + meta generation (write-sog.ts:110-370) and
// cluster1d (write-sog.ts:56-99), device-resident end to end.
//
// Order of work and of Math.random consumption follows writeSog exactly:
// Morton order -> means_l/u -> quats -> cluster1d(scales) -> cluster1d(f_dc)
// + opacity -> kmeans(SH, paletteSize) -> cluster1d(centroids) -> shN
// textures.  Texels beyond n stay zero (the reference's zero-initialised
// Uint8Arrays).  WebP encoding / ZIP packaging stay on the host (out of the
// device pipeline).
#include <cmath>
#include <exception>
#include <thread>

#include "st_jsmath.h"
#include "st_kmeans.h"
#include "st_typed.h"

namespace st {
namespace {

using namespace km;

__global__ __launch_bounds__(256) void k_concat1d(const float *const *cols, int ncols, uint64_t n, float *out) {
    const uint64_t total = n * (uint64_t)ncols;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride)
        out[i] = cols[i / n][i % n];
}

__global__ void k_sort_codebook(const float *cen, uint32_t *keys, uint32_t *vals) {
    const int i = threadIdx.x;
    keys[i] = sortkey_(cen[i]);
    vals[i] = (uint32_t)i;
}

__global__ void k_finish_codebook(const float *cen, const uint32_t *order, float *sorted, uint32_t *inv) {
    const int i = threadIdx.x;
    sorted[i] = cen[order[i]];
    inv[order[i]] = (uint32_t)i;
}

__global__ __launch_bounds__(256) void k_remap_labels(const uint32_t *lab, const uint32_t *inv, uint64_t total,
                                                      uint8_t *out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride)
        out[i] = (uint8_t)inv[lab[i]];
}


template <typename T>
struct MeansArgs {
    const T *c[3];
    double mn[3], mx[3];
};

// pos[idx[i]] = i: the texel of each row under the Morton order idx
__global__ __launch_bounds__(256) void k_invert(const uint32_t *__restrict__ idx, uint64_t n, uint32_t *__restrict__ pos) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        pos[idx[i]] = (uint32_t)i;
}

// Texture kernels run in two forms: gather (texel i <- row idx[i], the single-device
// writeSog) or scatter (local row i -> texel pos[i], one shard of a multi-GPU writeSog)
__device__ inline void tex_slot(const uint32_t *idx, const uint32_t *pos, uint64_t i, uint32_t &row, uint64_t &o) {
    row = pos ? (uint32_t)i : idx ? idx[i] : (uint32_t)i;  // neither: row order
    o = pos ? (uint64_t)pos[i] : i;
}

template <typename T>
__global__ __launch_bounds__(256) void k_means_tex(const MeansArgs<T> a, const uint32_t *__restrict__ idx,
                                                  const uint32_t *__restrict__ pos, uint64_t n,
                                                  uint32_t *__restrict__ ml, uint32_t *__restrict__ mu) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint32_t r;
        uint64_t o;
        tex_slot(idx, pos, i, r, o);
        uint32_t lw = 0xff000000u, up = 0xff000000u;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const double v = 65535 * (js::log_transform((double)a.c[k][r]) - a.mn[k]) / (a.mx[k] - a.mn[k]);
            const int32_t iv = js::to_int32(v);
            lw |= (uint32_t)(iv & 0xff) << (8 * k);
            up |= (uint32_t)((iv >> 8) & 0xff) << (8 * k);
        }
        ml[o] = lw;
        mu[o] = up;
    }
}

template <typename T>
__global__ __launch_bounds__(256) void k_quats_tex(const T *__restrict__ q0, const T *__restrict__ q1,
                                                  const T *__restrict__ q2, const T *__restrict__ q3,
                                                  const uint32_t *__restrict__ idx, const uint32_t *__restrict__ pos,
                                                  uint64_t n, uint32_t *__restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint32_t r;
        uint64_t o;
        tex_slot(idx, pos, i, r, o);
        double q[4] = {q0[r], q1[r], q2[r], q3[r]};
        const double l = __builtin_sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
#pragma unroll
        for (int j = 0; j < 4; ++j) q[j] = q[j] / l;
        int mc = 0;
#pragma unroll
        for (int j = 1; j < 4; ++j)
            if (__builtin_fabs(q[j]) > __builtin_fabs(q[mc])) mc = j;
        if (q[mc] < 0) {
#pragma unroll
            for (int j = 0; j < 4; ++j) q[j] *= -1;
        }
        const double sqrt2 = __builtin_sqrt(2.0);
#pragma unroll
        for (int j = 0; j < 4; ++j) q[j] *= sqrt2;
        uint32_t px = (uint32_t)(252 + mc) << 24;
        int k = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (j == mc) continue;
            px |= (uint32_t)js::to_uint8(255 * (q[j] * 0.5 + 0.5)) << (8 * k);
            ++k;
        }
        out[o] = px;
    }
}

// writeTableData (write-sog.ts:142-157): rgb from u8 label columns, alpha = 4th column or 255
template <typename T>
__global__ __launch_bounds__(256) void k_table_tex(const uint8_t *__restrict__ l0, const uint8_t *__restrict__ l1,
                                                  const uint8_t *__restrict__ l2, const T *__restrict__ opacity,
                                                  const uint32_t *__restrict__ idx, const uint32_t *__restrict__ pos,
                                                  uint64_t n, uint32_t *__restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint32_t r;
        uint64_t o;
        tex_slot(idx, pos, i, r, o);
        uint32_t a = 255;
        if (opacity) a = js::to_uint8(js::max_(0, js::min_(255, js::sigmoid((double)opacity[r]) * 255)));
        out[o] = (uint32_t)l0[r] | ((uint32_t)l1[r] << 8) | ((uint32_t)l2[r] << 16) | (a << 24);
    }
}

__global__ __launch_bounds__(256) void k_shn_labels_tex(const uint32_t *__restrict__ labels,
                                                       const uint32_t *__restrict__ idx,
                                                       const uint32_t *__restrict__ pos, uint64_t n,
                                                       uint32_t *__restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint32_t r;
        uint64_t o;
        tex_slot(idx, pos, i, r, o);
        const uint32_t label = labels[r];
        out[o] = (label & 0xffu) | (((label >> 8) & 0xffu) << 8) | 0xff000000u;
    }
}

// shN_centroids (write-sog.ts:319-335): centroid i, coefficient j -> texel i*C + j
__global__ __launch_bounds__(256) void k_shn_centroids_tex(const uint8_t *__restrict__ cl, int C, int pal,
                                                          uint32_t *__restrict__ out) {
    const uint64_t total = (uint64_t)pal * C;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
        const uint64_t i = t / C, j = t % C;
        out[t] = (uint32_t)cl[j * pal + i] | ((uint32_t)cl[(C + j) * pal + i] << 8) |
                 ((uint32_t)cl[(2 * C + j) * pal + i] << 16) | 0xff000000u;
    }
}

// calcMinMax (write-sog.ts:15-31) of float64 columns: NaN-ignoring min / max as ordered keys,
// one atomic per block and column
__device__ inline unsigned long long dkey(double d) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, d);
    return (u >> 63) ? ~u : (u | (1ull << 63));
}
__host__ inline double dkey_inv(unsigned long long k) {
    return __builtin_bit_cast(double, (k >> 63) ? (k & ~(1ull << 63)) : ~k);
}
__global__ __launch_bounds__(256) void k_mm64(const double *__restrict__ a, const double *__restrict__ b,
                                              const double *__restrict__ cc, uint64_t n,
                                              unsigned long long *__restrict__ out) {
    const double *cols[3] = {a, b, cc};
    unsigned long long mn[3] = {~0ull, ~0ull, ~0ull}, mx[3] = {0, 0, 0};
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        for (int q = 0; q < 3; ++q) {
            const double v = cols[q][i];
            if (v == v) {
                const unsigned long long k = dkey(v);
                mn[q] = k < mn[q] ? k : mn[q];
                mx[q] = k > mx[q] ? k : mx[q];
            }
        }
    for (int q = 0; q < 3; ++q) {
        for (int o = 32; o > 0; o >>= 1) {
            const unsigned long long t0 = __shfl_xor(mn[q], o, 64), t1 = __shfl_xor(mx[q], o, 64);
            mn[q] = t0 < mn[q] ? t0 : mn[q];
            mx[q] = t1 > mx[q] ? t1 : mx[q];
        }
        if ((threadIdx.x & 63) == 0) {
            if (mn[q] != ~0ull) atomicMin(&out[2 * q], mn[q]);
            if (mx[q] != 0ull) atomicMax(&out[2 * q + 1], mx[q]);
        }
    }
}

int palette_of(uint64_t n) {
    int lg = 0;
    while ((2ull << lg) <= n) ++lg;  // floor(log2 n)
    const int p = lg - 10;           // floor(log2(n / 1024))
    if (p >= 6) return 64 * 1024;
    if (p >= 0) return (1 << p) * 1024;
    return 1024 >> (-p);
}

}  // namespace

uint64_t cluster1d_dev(st_ctx *c, const float *const *cols, int ncols, uint64_t n, int iters, const double *draws,
                       uint64_t ndraws, float *centroids256, uint8_t *labels) {
    const uint64_t total = n * (uint64_t)ncols;
    ST_REQUIRE(total >= 256, ST_ERR_ARG,
               "cluster1d: fewer than 256 values (the reference's kmeans returns a plain Array and .subarray throws)");
    auto **dcols = wsT<const float *>(c, "c1.cols", (size_t)ncols);
    ST_HIP(hipMemcpyAsync(dcols, cols, sizeof(float *) * ncols, hipMemcpyHostToDevice, c->stream));
    auto *data = wsT<float>(c, "c1.data", total);
    hipLaunchKernelGGL(k_concat1d, dim3(grid_for(total, 256, 8192)), dim3(256), 0, c->stream, dcols, ncols, n, data);
    ST_LAUNCH_CHECK();
    auto *cen = wsT<float>(c, "c1.cen", 256);
    auto *lab = wsT<uint32_t>(c, "c1.lab", total);
    const float *one[1] = {data};
    const uint64_t used = kmeans_dev(c, one, 1, total, 256, iters, draws, ndraws, cen, lab);
    codebook_dev(c, cen, lab, total, centroids256, labels);
    return used;
}

// cluster1d's codebook (write-sog.ts:69-88): centroids sorted ascending (stable,
// `a - b` comparator), labels remapped to the sorted order as bytes
void codebook_dev(st_ctx *c, const float *cen, const uint32_t *lab, uint64_t total, float *centroids256,
                  uint8_t *labels) {
    auto *keys = wsT<uint32_t>(c, "c1.keys", 256);
    auto *order = wsT<uint32_t>(c, "c1.order", 256);
    auto *inv = wsT<uint32_t>(c, "c1.inv", 256);
    hipLaunchKernelGGL(k_sort_codebook, dim3(1), dim3(256), 0, c->stream, cen, keys, order);
    radix_sort_u32(c, keys, order, 256, 0, 32, "c1.rs");
    hipLaunchKernelGGL(k_finish_codebook, dim3(1), dim3(256), 0, c->stream, cen, order, centroids256, inv);
    if (total)
        hipLaunchKernelGGL(k_remap_labels, dim3(grid_for(total, 256, 8192)), dim3(256), 0, c->stream, lab, inv, total,
                           labels);
    ST_LAUNCH_CHECK();
}

// one shard's texels of a multi-GPU writeSog: local rows at their global sorted
// positions `pos`; lo/hi are the global NaN-ignoring extents of x, y, z
void sog_scatter_dev(st_ctx *c, const st_table *t, const uint32_t *pos, const double lo[3], const double hi[3],
                     const uint8_t *scale_lab, const uint8_t *color_lab, const uint32_t *shn_lab, st_sog_meta *meta,
                     const st_sog_textures *out) {
    const uint64_t n = t->n;
    static const char *members[8] = {"x", "y", "z", "opacity", "rot_0", "rot_1", "rot_2", "rot_3"};
    const float *m[8];
    for (int i = 0; i < 8; ++i) {
        m[i] = col_or_null(t, members[i]);
        // an empty shard's columns may be NULL (no rows to read): only the meta is computed
        ST_REQUIRE(m[i] || n == 0, ST_ERR_ARG, std::string("sog: missing column ") + members[i]);
    }
    MeansArgs<float> ma{};
    for (int a = 0; a < 3; ++a) {
        ma.c[a] = m[a];
        ma.mn[a] = js::log_transform(lo[a]);
        ma.mx[a] = js::log_transform(hi[a]);
        meta->means_min[a] = ma.mn[a];
        meta->means_max[a] = ma.mx[a];
    }
    if (!n) return;
    const unsigned g = grid_for(n, 256, 8192);
    if (out->means_l && out->means_u)
        hipLaunchKernelGGL(k_means_tex<float>, dim3(g), dim3(256), 0, c->stream, ma, (const uint32_t *)nullptr, pos, n,
                           (uint32_t *)out->means_l, (uint32_t *)out->means_u);
    if (out->quats)
        hipLaunchKernelGGL(k_quats_tex<float>, dim3(g), dim3(256), 0, c->stream, m[4], m[5], m[6], m[7],
                           (const uint32_t *)nullptr, pos, n, (uint32_t *)out->quats);
    if (out->scales && scale_lab)
        hipLaunchKernelGGL(k_table_tex<float>, dim3(g), dim3(256), 0, c->stream, scale_lab, scale_lab + n, scale_lab + 2 * n,
                           (const float *)nullptr, (const uint32_t *)nullptr, pos, n, (uint32_t *)out->scales);
    if (out->sh0 && color_lab)
        hipLaunchKernelGGL(k_table_tex<float>, dim3(g), dim3(256), 0, c->stream, color_lab, color_lab + n, color_lab + 2 * n,
                           m[3], (const uint32_t *)nullptr, pos, n, (uint32_t *)out->sh0);
    if (out->shn_labels && shn_lab)
        hipLaunchKernelGGL(k_shn_labels_tex, dim3(g), dim3(256), 0, c->stream, shn_lab, (const uint32_t *)nullptr,
                           pos, n, (uint32_t *)out->shn_labels);
    ST_LAUNCH_CHECK();
}

// the scales / sh0 texels (write-sog.ts:245-268) of n rows in row order: out[r] from the byte labels
// lab[0..3n) (three planes) and the opacity (nullable: alpha 255)
void sog_table_rows(st_ctx *c, uint64_t n, const uint8_t *lab, const float *opacity, uint8_t *out) {
    if (!n) return;
    hipLaunchKernelGGL(k_table_tex<float>, dim3(grid_for(n, 256, 8192)), dim3(256), 0, c->stream, lab, lab + n,
                       lab + 2 * n, opacity, (const uint32_t *)nullptr, (const uint32_t *)nullptr, n, (uint32_t *)out);
    ST_LAUNCH_CHECK();
}

// cluster1d of the scales (a) then of the colours (b), write-sog.ts:245-268, as sog_impl runs
// them: b on the context `side` from its own host thread, from draw 0 (re-seeds of empty
// clusters are the only draws a 1-D k-means takes, and b's come after a's), kept when a took no
// draw and otherwise rerun here at a's cursor.  Returns the draws both took.
uint64_t cluster1d_pair_dev(st_ctx *c, st_ctx *side, const float *const *a, const float *const *b, uint64_t n,
                            int iters, const double *draws, uint64_t ndraws, float *cb_a, uint8_t *lab_a, float *cb_b,
                            uint8_t *lab_b) {
    {
        hipEvent_t ev;  // the columns: whatever the caller queued on c->stream first
        ST_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        ST_HIP(hipEventRecord(ev, c->stream));
        ST_HIP(hipStreamWaitEvent(side->stream, ev, 0));
        ST_HIP(hipEventDestroy(ev));
    }
    uint64_t used_b = 0;
    std::exception_ptr err_b;
    std::thread th([&] {
        try {
            use_device(side);
            used_b = cluster1d_dev(side, b, 3, n, iters, draws, ndraws, cb_b, lab_b);
            ST_HIP(hipStreamSynchronize(side->stream));
        } catch (...) {
            err_b = std::current_exception();
        }
    });
    struct Join {
        std::thread &t;
        ~Join() {
            if (t.joinable()) t.join();
        }
    } join{th};
    const uint64_t used_a = cluster1d_dev(c, a, 3, n, iters, draws, ndraws, cb_a, lab_a);
    th.join();
    if (used_a == 0) {
        if (err_b) std::rethrow_exception(err_b);
        return used_b;
    }
    return used_a + cluster1d_dev(c, b, 3, n, iters, draws + used_a, ndraws - used_a, cb_b, lab_b);
}

void shn_centroids_dev(st_ctx *c, const uint8_t *cl, int C, int pal, uint8_t *out) {
    hipLaunchKernelGGL(k_shn_centroids_tex, dim3(grid_for((uint64_t)pal * C, 256, 4096)), dim3(256), 0, c->stream,
                       cl, C, pal, (uint32_t *)out);
    ST_LAUNCH_CHECK();
}

namespace {
const char *const SOG_MEMBERS[14] = {"x", "y", "z", "scale_0", "scale_1", "scale_2", "f_dc_0",
                                     "f_dc_1", "f_dc_2", "opacity", "rot_0", "rot_1", "rot_2", "rot_3"};

// the columns writeSog reads: Float32Array values (cluster1d data, k-means points) and, where a
// column is not float32, the JS numbers the reference computes with (positions, rotations,
// opacity, and the SH values calcAverage sums)
struct SogSrc {
    uint64_t n = 0;
    int C = 0;
    const float *m[14] = {};
    const double *pos64[3] = {};  // all three set or none
    const double *rot64[4] = {};  // all four set or none
    const double *op64 = nullptr;
    const float *sh[45] = {};
    const double *sh64[45] = {};  // all 3C set or none
};

uint64_t sog_impl(st_ctx *c, const SogSrc &src, int iters, const double *draws, uint64_t ndraws,
                  st_sog_meta *meta, const st_sog_textures *out);
}  // namespace

uint64_t sog_dev(st_ctx *c, const st_table *t, int iters, const double *draws, uint64_t ndraws, st_sog_meta *meta,
                 const st_sog_textures *out) {
    SogSrc src;
    src.n = t->n;
    for (int i = 0; i < 14; ++i) {
        src.m[i] = col_or_null(t, SOG_MEMBERS[i]);
        ST_REQUIRE(src.m[i], ST_ERR_ARG, std::string("sog: missing column ") + SOG_MEMBERS[i]);
    }
    src.C = sh_coeffs_of(t);
    char nm[32];
    for (int i = 0; i < 3 * src.C; ++i) {
        snprintf(nm, sizeof nm, "f_rest_%d", i);
        src.sh[i] = col_or_null(t, nm);
    }
    return sog_impl(c, src, iters, draws, ndraws, meta, out);
}

uint64_t sog_tdev(st_ctx *c, const st_ttable *t, int iters, const double *draws, uint64_t ndraws,
                  st_sog_meta *meta, const st_sog_textures *out) {
    SogSrc src;
    src.n = t->n;
    TCol tc[14];
    for (int i = 0; i < 14; ++i) {
        tc[i] = tcol_or_null(t, SOG_MEMBERS[i]);
        ST_REQUIRE(tc[i].p, ST_ERR_ARG, std::string("sog: missing column ") + SOG_MEMBERS[i]);
        src.m[i] = as_f32_dev(c, tc[i], src.n, "sogt.m32." + std::to_string(i));
    }
    const auto f64 = [&](int i) { return as_f64_dev(c, tc[i], src.n, "sogt.m64." + std::to_string(i)); };
    if (tc[0].t != ST_PLY_FLOAT || tc[1].t != ST_PLY_FLOAT || tc[2].t != ST_PLY_FLOAT)
        for (int a = 0; a < 3; ++a) src.pos64[a] = f64(a);
    if (tc[10].t != ST_PLY_FLOAT || tc[11].t != ST_PLY_FLOAT || tc[12].t != ST_PLY_FLOAT || tc[13].t != ST_PLY_FLOAT)
        for (int a = 0; a < 4; ++a) src.rot64[a] = f64(10 + a);
    if (tc[9].t != ST_PLY_FLOAT) src.op64 = f64(9);
    int first_missing = -1;
    char nm[32];
    for (int i = 0; i < 45 && first_missing < 0; ++i) {
        snprintf(nm, sizeof nm, "f_rest_%d", i);
        if (!tcol_or_null(t, nm).p) first_missing = i;
    }
    src.C = first_missing == 9 ? 3 : first_missing == 24 ? 8 : first_missing == -1 ? 15 : 0;
    bool sh32 = true;
    for (int i = 0; i < 3 * src.C; ++i) {
        snprintf(nm, sizeof nm, "f_rest_%d", i);
        const TCol col = tcol_or_null(t, nm);
        sh32 = sh32 && col.t == ST_PLY_FLOAT;
        src.sh[i] = as_f32_dev(c, col, src.n, "sogt.sh32." + std::to_string(i));
    }
    if (!sh32)
        for (int i = 0; i < 3 * src.C; ++i) {
            snprintf(nm, sizeof nm, "f_rest_%d", i);
            src.sh64[i] = as_f64_dev(c, tcol_or_null(t, nm), src.n, "sogt.sh64." + std::to_string(i));
        }
    return sog_impl(c, src, iters, draws, ndraws, meta, out);
}

namespace {
uint64_t sog_impl(st_ctx *c, const SogSrc &src, int iters, const double *draws, uint64_t ndraws,
                  st_sog_meta *meta, const st_sog_textures *out) {
    const uint64_t n = src.n;
    ST_REQUIRE(n > 0, ST_ERR_ARG, "sog: empty table");
    ST_REQUIRE(n < (1ull << 31), ST_ERR_ARG, "sog: n must be < 2^31 per device");
    const float *const *m = src.m;
    const int C = src.C;
    int32_t W, H, pal, cw, chh;
    st_sog_geometry(n, C, &W, &H, &pal, &cw, &chh);
    const uint64_t texels = (uint64_t)W * H;
    *meta = st_sog_meta{};
    meta->width = W;
    meta->height = H;
    for (uint8_t *p : {out->means_l, out->means_u, out->quats, out->scales, out->sh0})
        ST_REQUIRE(p, ST_ERR_ARG, "sog: texture output is NULL");
    for (uint8_t *p : {out->means_l, out->means_u, out->quats, out->scales, out->sh0})
        ST_HIP(hipMemsetAsync(p, 0, texels * 4, c->stream));

    // cluster1d of the colours (write-sog.ts:253-268) runs on a side context from its own host
    // thread while this one orders, packs means / quats and clusters the scales.  Its draws
    // start where the scales' k-means stops taking them (re-seeds of empty clusters only), so
    // it starts at the scales' cursor 0 and is kept only if the scales took no draw; otherwise
    // it reruns here at the right cursor (bit-identical either way)
    if (!c->aux) ST_REQUIRE(st_ctx_create(c->device, &c->aux) == ST_OK, ST_ERR_HIP, "sog: side context");
    st_ctx *aux = c->aux;
    auto *lab_c = wsT<uint8_t>(aux, "sog.lab_c", n * 3);
    auto *cb_c = wsT<float>(aux, "sog.cb_c", 256);
    uint64_t used_c = 0;
    std::exception_ptr err_c;
    {
        // the colour columns are the caller's: whatever the caller queued on c->stream first
        hipEvent_t ev;
        ST_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        ST_HIP(hipEventRecord(ev, c->stream));
        ST_HIP(hipStreamWaitEvent(aux->stream, ev, 0));
        ST_HIP(hipEventDestroy(ev));
    }
    std::thread colours([&] {
        try {
            use_device(aux);
            used_c = cluster1d_dev(aux, m + 6, 3, n, iters, draws, ndraws, cb_c, lab_c);
            ST_HIP(hipStreamSynchronize(aux->stream));
        } catch (...) {
            err_c = std::current_exception();
        }
    });
    struct Joiner {
        std::thread &th;
        ~Joiner() {
            if (th.joinable()) th.join();
        }
    } joiner{colours};

    // Morton order, extents and the five textures on a third context from their own host
    // thread (c->aux->aux), started once both cluster1d are done so that the 1-D block runs
    // alone and the Morton passes overlap the SH k-means' sweep instead: only the shN texture
    // writes wait for the texel positions
    auto *pos = wsT<uint32_t>(c, "sog.pos", n);
    const unsigned g = grid_for(n, 256, 8192);
    if (!aux->aux) ST_REQUIRE(st_ctx_create(c->device, &aux->aux) == ST_OK, ST_ERR_HIP, "sog: side context");
    st_ctx *mc = aux->aux;
    hipEvent_t ev_pos, ev_lab;
    ST_HIP(hipEventCreateWithFlags(&ev_pos, hipEventDisableTiming));
    ST_HIP(hipEventCreateWithFlags(&ev_lab, hipEventDisableTiming));
    {
        hipEvent_t ev;  // the textures' clears above and the caller's columns
        ST_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        ST_HIP(hipEventRecord(ev, c->stream));
        ST_HIP(hipStreamWaitEvent(mc->stream, ev, 0));
        ST_HIP(hipEventDestroy(ev));
    }
    std::exception_ptr err_m;
    const uint8_t *lab_s_ = nullptr, *clab_ = nullptr;  // the labels the texture writes read
    auto order_fn = [&] {
        try {
            use_device(mc);
            // Morton order (write-sog.ts:42-49)
            auto *idx = wsT<uint32_t>(mc, "sog.idx", n);
            iota_u32(mc, idx, n);
            if (src.pos64[0]) morton_order_dev_f64(mc, src.pos64[0], src.pos64[1], src.pos64[2], idx, n);
            else morton_order_dev(mc, m[0], m[1], m[2], idx, n);
            // the texture kernels run in scatter form: row r (read in input order, coalesced) writes
            // texel pos[r], one 4-byte store, instead of gathering 3-4 values per texel at random
            hipLaunchKernelGGL(k_invert, dim3(grid_for(n, 256, 8192)), dim3(256), 0, mc->stream, idx, n, pos);
            ST_LAUNCH_CHECK();

            // means (write-sog.ts:161-187)
            double lo[3], hi[3];
            if (src.pos64[0]) {
                auto *mm = wsT<unsigned long long>(mc, "sog.mm64", 6);
                const unsigned long long init[6] = {~0ull, 0ull, ~0ull, 0ull, ~0ull, 0ull};
                unsigned long long hmm[6];
                ST_HIP(hipMemcpyAsync(mm, init, sizeof init, hipMemcpyHostToDevice, mc->stream));
                hipLaunchKernelGGL(k_mm64, dim3(grid_for(n, 256, 1024)), dim3(256), 0, mc->stream, src.pos64[0], src.pos64[1],
                                   src.pos64[2], n, mm);
                ST_LAUNCH_CHECK();
                ST_HIP(hipMemcpyAsync(hmm, mm, sizeof hmm, hipMemcpyDeviceToHost, mc->stream));
                ST_HIP(hipStreamSynchronize(mc->stream));
                for (int a = 0; a < 3; ++a) {
                    lo[a] = hmm[2 * a] == ~0ull ? HUGE_VAL : dkey_inv(hmm[2 * a]);
                    hi[a] = hmm[2 * a + 1] == 0ull ? -HUGE_VAL : dkey_inv(hmm[2 * a + 1]);
                }
            } else {
                auto *mm = wsT<uint32_t>(mc, "sog.mm", 6);
                minmax_keys_dev(mc, m, 3, n, mm);  // [min, max] keys of x, y, z (NaN skipped)
                uint32_t hmm[6];
                ST_HIP(hipMemcpyAsync(hmm, mm, sizeof hmm, hipMemcpyDeviceToHost, mc->stream));
                ST_HIP(hipStreamSynchronize(mc->stream));
                for (int a = 0; a < 3; ++a) {
                    lo[a] = hmm[2 * a] == 0xffffffffu ? HUGE_VAL : (double)fkey_inv_(hmm[2 * a]);
                    hi[a] = hmm[2 * a + 1] == 0u ? -HUGE_VAL : (double)fkey_inv_(hmm[2 * a + 1]);
                }
            }
            for (int a = 0; a < 3; ++a) {
                meta->means_min[a] = js::log_transform(lo[a]);
                meta->means_max[a] = js::log_transform(hi[a]);
            }
            if (src.pos64[0]) {
                MeansArgs<double> ma{};
                for (int a = 0; a < 3; ++a) ma.c[a] = src.pos64[a], ma.mn[a] = meta->means_min[a], ma.mx[a] = meta->means_max[a];
                hipLaunchKernelGGL(k_means_tex<double>, dim3(g), dim3(256), 0, mc->stream, ma, (const uint32_t *)nullptr, pos,
                                   n, (uint32_t *)out->means_l, (uint32_t *)out->means_u);
            } else {
                MeansArgs<float> ma{};
                for (int a = 0; a < 3; ++a) ma.c[a] = m[a], ma.mn[a] = meta->means_min[a], ma.mx[a] = meta->means_max[a];
                hipLaunchKernelGGL(k_means_tex<float>, dim3(g), dim3(256), 0, mc->stream, ma, (const uint32_t *)nullptr, pos, n,
                                   (uint32_t *)out->means_l, (uint32_t *)out->means_u);
            }
            if (src.rot64[0])
                hipLaunchKernelGGL(k_quats_tex<double>, dim3(g), dim3(256), 0, mc->stream, src.rot64[0], src.rot64[1],
                                   src.rot64[2], src.rot64[3], (const uint32_t *)nullptr, pos, n, (uint32_t *)out->quats);
            else
                hipLaunchKernelGGL(k_quats_tex<float>, dim3(g), dim3(256), 0, mc->stream, m[10], m[11], m[12], m[13],
                                   (const uint32_t *)nullptr, pos, n, (uint32_t *)out->quats);
            ST_LAUNCH_CHECK();
            {  // the scales / sh0 texels, once the labels are in place
                ST_HIP(hipStreamWaitEvent(mc->stream, ev_lab, 0));
                hipLaunchKernelGGL(k_table_tex<float>, dim3(g), dim3(256), 0, mc->stream, lab_s_, lab_s_ + n, lab_s_ + 2 * n,
                                   (const float *)nullptr, (const uint32_t *)nullptr, pos, n, (uint32_t *)out->scales);
                if (src.op64)
                    hipLaunchKernelGGL(k_table_tex<double>, dim3(g), dim3(256), 0, mc->stream, clab_, clab_ + n,
                                       clab_ + 2 * n, src.op64, (const uint32_t *)nullptr, pos, n, (uint32_t *)out->sh0);
                else
                    hipLaunchKernelGGL(k_table_tex<float>, dim3(g), dim3(256), 0, mc->stream, clab_, clab_ + n,
                                       clab_ + 2 * n, m[9], (const uint32_t *)nullptr, pos, n, (uint32_t *)out->sh0);
                ST_LAUNCH_CHECK();
            }
            ST_HIP(hipEventRecord(ev_pos, mc->stream));
            if (c->sog_early) c->sog_early(mc);  // the five textures are final on mc->stream
            ST_HIP(hipStreamSynchronize(mc->stream));
        } catch (...) {
            err_m = std::current_exception();
        }
    };
    std::thread order_th;
    struct Joiner2 {
        std::thread &th;
        hipEvent_t ev, ev2;
        ~Joiner2() {
            if (th.joinable()) th.join();
            (void)hipEventDestroy(ev);
            (void)hipEventDestroy(ev2);
        }
    } joiner2{order_th, ev_pos, ev_lab};

    uint64_t cursor = 0;
    auto *lab = wsT<uint8_t>(c, "sog.lab", n * 3);
    auto *cb = wsT<float>(c, "sog.cb", 256);
    // scales (write-sog.ts:245-251)
    cursor += cluster1d_dev(c, m + 3, 3, n, iters, draws + cursor, ndraws - cursor, cb, lab);
    ST_HIP(hipMemcpyAsync(meta->scales_codebook, cb, 256 * 4, hipMemcpyDeviceToHost, c->stream));
    // colour + opacity (write-sog.ts:253-268)
    colours.join();
    const uint8_t *clab = lab_c;
    const float *ccb = cb_c;
    uint8_t *lab_s = lab;
    if (cursor == 0) {
        if (err_c) std::rethrow_exception(err_c);
        cursor += used_c;
    } else {  // the scales took draws: the colours' k-means starts after them
        lab_s = wsT<uint8_t>(c, "sog.lab_s", n * 3);
        ST_HIP(hipMemcpyAsync(lab_s, lab, n * 3, hipMemcpyDeviceToDevice, c->stream));
        cursor += cluster1d_dev(c, m + 6, 3, n, iters, draws + cursor, ndraws - cursor, cb, lab);
        clab = lab;
        ccb = cb;
    }
    ST_HIP(hipMemcpyAsync(meta->sh0_codebook, ccb, 256 * 4, hipMemcpyDeviceToHost, c->stream));
    mark(c, "sog.cluster1d");
    // the Morton order and the five textures beside the SH k-means (order_fn)
    lab_s_ = lab_s;
    clab_ = clab;
    ST_HIP(hipEventRecord(ev_lab, c->stream));
    if (c->sog_early && !mc->aux)
        ST_REQUIRE(st_ctx_create(c->device, &mc->aux) == ST_OK, ST_ERR_HIP, "sog: side context");
    order_th = std::thread(order_fn);
    // the texture thread ends before anything reads the texel positions on this stream
    auto join_late = [&] {
        if (!order_th.joinable()) return;
        order_th.join();
        if (err_m) std::rethrow_exception(err_m);
        ST_HIP(hipStreamWaitEvent(c->stream, ev_pos, 0));
    };

    meta->sh_bands = C == 15 ? 3 : C == 8 ? 2 : C == 3 ? 1 : 0;
    if (C > 0) {
        ST_REQUIRE(out->shn_centroids && out->shn_labels, ST_ERR_ARG, "sog: shN texture outputs are NULL");
        meta->palette_size = pal;
        meta->shn_width = cw;
        meta->shn_height = chh;
        const int D = 3 * C;
        auto *cen = wsT<float>(c, "sog.shcen", (size_t)pal * D);
        auto *labels = wsT<uint32_t>(c, "sog.shlab", n);
        cursor += kmeans_dev(c, src.sh, D, n, pal, iters, draws + cursor, ndraws - cursor, cen, labels, false,
                             src.sh64[0] ? src.sh64 : nullptr);
        mark(c, "sog.shkmeans");
        join_late();
        // the shN labels texels (random 4-byte stores at the Morton positions) do not wait for
        // the codebook: they run on the side stream beside its latency-bound 1-D iterations,
        // on few workgroups so that those kernels still find free CUs
        const hipStream_t ss = side_stream(c);
        ST_HIP(hipEventRecord(c->side_ev[0], c->stream));
        ST_HIP(hipStreamWaitEvent(ss, c->side_ev[0], 0));
        ST_HIP(hipMemsetAsync(out->shn_labels, 0, texels * 4, ss));
        // one workgroup per CU: the rest of each CU stays free for the codebook's kernels
        hipLaunchKernelGGL(k_shn_labels_tex, dim3(std::min(g, 256u)), dim3(256), 0, ss, labels,
                           (const uint32_t *)nullptr, pos, n, (uint32_t *)out->shn_labels);
        ST_LAUNCH_CHECK();
        ST_HIP(hipEventRecord(c->side_ev[1], ss));
        std::vector<const float *> ccols(D);
        for (int i = 0; i < D; ++i) ccols[i] = cen + (uint64_t)i * pal;
        auto *cl = wsT<uint8_t>(c, "sog.cl", (size_t)pal * D);
        try {
            // the SH centroids are initial rows, means of finite rows or re-seeded rows: finite
            c->km_finite_known = true;
            cursor += cluster1d_dev(c, ccols.data(), D, (uint64_t)pal, iters, draws + cursor, ndraws - cursor, cb, cl);
            c->km_finite_known = false;
        } catch (...) {
            c->km_finite_known = false;
            (void)hipStreamWaitEvent(c->stream, c->side_ev[1], 0);
            throw;
        }
        ST_HIP(hipMemcpyAsync(meta->shn_codebook, cb, 256 * 4, hipMemcpyDeviceToHost, c->stream));
        ST_HIP(hipMemsetAsync(out->shn_centroids, 0, (size_t)cw * chh * 4, c->stream));
        hipLaunchKernelGGL(k_shn_centroids_tex, dim3(grid_for((uint64_t)pal * C, 256, 4096)), dim3(256), 0, c->stream,
                           cl, C, pal, (uint32_t *)out->shn_centroids);
        ST_LAUNCH_CHECK();
        ST_HIP(hipStreamWaitEvent(c->stream, c->side_ev[1], 0));
        mark(c, "sog.shn");
    }
    join_late();
    ST_HIP(hipStreamSynchronize(c->stream));
    return cursor;
}
}  // namespace

}  // namespace st

extern "C" int st_sog_geometry(uint64_t n, int32_t C, int32_t *w, int32_t *h, int32_t *pal, int32_t *cw,
                               int32_t *ch) {
    if (n == 0) return ST_ERR_ARG;
    const int W = (int)(std::ceil(std::sqrt((double)n) / 4) * 4);
    const int H = (int)(std::ceil((double)n / W / 4) * 4);
    const int P = C > 0 ? st::palette_of(n) : 0;
    if (w) *w = W;
    if (h) *h = H;
    if (pal) *pal = P;
    if (cw) *cw = 64 * C;
    if (ch) *ch = C > 0 ? (P + 63) / 64 : 0;
    return ST_OK;
}
