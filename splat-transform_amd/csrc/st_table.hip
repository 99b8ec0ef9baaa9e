// st_table.hip -- the reference's whole-table row operations on typed SoA columns:
//   filterNaN   process.ts:84-95 (+ filter :47-61): keep a row iff every column value
//               isFinite -- float32 and float64 columns are tested, integer columns are
//               always finite
//   permuteRows data-table.ts:135-149: dst[c][j] = src[c][idx[j]] for every column type
//   combine     index.ts:158-210: columns united by (name, dataType) in first-seen order,
//               rows appended in table order, absent columns zero-filled
// Column types are st_ply_type codes (the reference's eight TypedArrays).  4-byte columns
// take the wide streaming kernels (4 rows per thread, 8 columns' loads in flight); 1, 2 and
// 8-byte columns a per-size gather.  All HBM-bound.
#include <cstring>

#include "st_internal.h"
#include "st_jsmath.h"

namespace st {

int type_size(int32_t type) {
    switch (type) {
        case ST_PLY_CHAR: case ST_PLY_UCHAR: return 1;
        case ST_PLY_SHORT: case ST_PLY_USHORT: return 2;
        case ST_PLY_INT: case ST_PLY_UINT: case ST_PLY_FLOAT: return 4;
        case ST_PLY_DOUBLE: return 8;
        default: return 0;
    }
}

namespace {

// ---------------------------------------------------------------------------
// filterNaN: keep row iff every column value is finite (process.ts:84-95)
__global__ __launch_bounds__(256) void k_finite_flags(float *const *cols, int ncol, uint64_t n, uint32_t *flags) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint32_t ok = 1;
        for (int c = 0; c < ncol; ++c) ok &= js::isfinitef_(cols[c][i]) ? 1u : 0u;
        flags[i] = ok;
    }
}

__global__ __launch_bounds__(256) void k_compact(const uint32_t *flags, const uint32_t *pos, uint64_t n,
                                                 uint32_t *out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        if (flags[i]) out[pos[i]] = (uint32_t)i;
}

// filterByValue's predicate on one column (process.ts:99-106), in f64 like the JS comparison
template <typename T>
__global__ __launch_bounds__(256) void k_cmp_flags(const T *__restrict__ col, uint64_t n, int cmp, double v,
                                                   uint32_t *flags) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const double x = (double)col[i];
        bool keep;
        switch (cmp) {
            case ST_CMP_LT: keep = x < v; break;
            case ST_CMP_LTE: keep = x <= v; break;
            case ST_CMP_GT: keep = x > v; break;
            case ST_CMP_GTE: keep = x >= v; break;
            case ST_CMP_EQ: keep = x == v; break;
            default: keep = !(x == v); break;  // ST_CMP_NEQ: !== (true when either is NaN)
        }
        flags[i] = keep ? 1u : 0u;
    }
}

// permuteRows (data-table.ts:135-149): dst[c][j] = src[c][idx[j]]
__global__ __launch_bounds__(256) void k_gather_cols(float *const *src, float *const *dst, int ncol,
                                                     const uint32_t *__restrict__ idx, uint64_t m) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += stride) {
        const uint32_t s = idx[j];
        for (int c = 0; c < ncol; ++c) dst[c][j] = src[c][s];
    }
}

// ---- wide streaming forms: 4 consecutive rows per thread, column pointers in kernel
// arguments, 8 columns' loads in flight before any test (the loops above wait on every
// column's load in turn)
constexpr int WIDE_COLS = 64;
struct ColPtrs {
    const float *p[WIDE_COLS];
};

__device__ inline uint32_t nonfinite_bit(float x) {
    return ((__builtin_bit_cast(uint32_t, x) & 0x7f800000u) == 0x7f800000u) ? 1u : 0u;
}

__global__ __launch_bounds__(256) void k_finite_flags4(const ColPtrs cp, int ncol, uint64_t n,
                                                       uint32_t *__restrict__ flags) {
    const uint64_t nq = n / 4;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nq; q += stride) {
        uint32_t bad = 0;  // bit r: row 4q + r holds a non-finite value
        int c = 0;
        for (; c + 8 <= ncol; c += 8) {
            float4 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = reinterpret_cast<const float4 *>(cp.p[c + u])[q];
#pragma unroll
            for (int u = 0; u < 8; ++u)
                bad |= nonfinite_bit(v[u].x) | (nonfinite_bit(v[u].y) << 1) | (nonfinite_bit(v[u].z) << 2) |
                       (nonfinite_bit(v[u].w) << 3);
        }
        for (; c < ncol; ++c) {
            const float4 v = reinterpret_cast<const float4 *>(cp.p[c])[q];
            bad |= nonfinite_bit(v.x) | (nonfinite_bit(v.y) << 1) | (nonfinite_bit(v.z) << 2) | (nonfinite_bit(v.w) << 3);
        }
        reinterpret_cast<uint4 *>(flags)[q] =
            make_uint4((bad & 1u) ^ 1u, ((bad >> 1) & 1u) ^ 1u, ((bad >> 2) & 1u) ^ 1u, ((bad >> 3) & 1u) ^ 1u);
    }
    if (blockIdx.x == 0 && threadIdx.x < n % 4) {  // the last n % 4 rows
        const uint64_t i = nq * 4 + threadIdx.x;
        uint32_t bad = 0;
        for (int c = 0; c < ncol; ++c) bad |= nonfinite_bit(cp.p[c][i]);
        flags[i] = bad ^ 1u;
    }
}

// permuteRows with 4 destination rows per thread: 4 x 8 gathered loads in flight, float4
// stores (dst columns and idx 16-byte aligned)
__global__ __launch_bounds__(256) void k_gather_cols4(const ColPtrs src, const ColPtrs dst, int ncol,
                                                      const uint32_t *__restrict__ idx, uint64_t m) {
    const uint64_t mq = m / 4;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < mq; q += stride) {
        const uint4 ii = reinterpret_cast<const uint4 *>(idx)[q];
        int c = 0;
        for (; c + 8 <= ncol; c += 8) {
            float4 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const float *sp = src.p[c + u];
                v[u] = make_float4(sp[ii.x], sp[ii.y], sp[ii.z], sp[ii.w]);
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) reinterpret_cast<float4 *>(const_cast<float *>(dst.p[c + u]))[q] = v[u];
        }
        for (; c < ncol; ++c) {
            const float *sp = src.p[c];
            reinterpret_cast<float4 *>(const_cast<float *>(dst.p[c]))[q] =
                make_float4(sp[ii.x], sp[ii.y], sp[ii.z], sp[ii.w]);
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < m % 4) {
        const uint64_t j = mq * 4 + threadIdx.x;
        const uint32_t sj = idx[j];
        for (int c = 0; c < ncol; ++c) const_cast<float *>(dst.p[c])[j] = src.p[c][sj];
    }
}

bool aligned16(const void *p) { return ((uintptr_t)p & 15u) == 0; }


// float64 columns: flags[i] &= every f64 value of row i is finite
__global__ __launch_bounds__(256) void k_finite_and_f64(const double *const *cols, int ncol, uint64_t n,
                                                        uint32_t *flags) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint32_t ok = flags[i];
        for (int c = 0; c < ncol; ++c) {
            const uint64_t u = __builtin_bit_cast(uint64_t, cols[c][i]);
            ok &= ((u & 0x7ff0000000000000ull) != 0x7ff0000000000000ull) ? 1u : 0u;
        }
        flags[i] = ok;
    }
}

// permuteRows for 1, 2 and 8-byte columns (bit copies)
template <typename T>
__global__ __launch_bounds__(256) void k_gather_t(T *const *src, T *const *dst, int ncol,
                                                  const uint32_t *__restrict__ idx, uint64_t m) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += stride) {
        const uint32_t s = idx[j];
        for (int c = 0; c < ncol; ++c) dst[c][j] = src[c][s];
    }
}

}  // namespace

template <typename T>
static T *const *upload_ptrs(st_ctx *c, const std::string &slot, const std::vector<T *> &ptrs) {
    auto **d = wsT<T *>(c, slot, ptrs.size() ? ptrs.size() : 1);
    if (!ptrs.empty()) ST_HIP(hipMemcpyAsync(d, ptrs.data(), sizeof(T *) * ptrs.size(), hipMemcpyHostToDevice, c->stream));
    return d;
}

// flags[i] = 1 iff every float32 column is finite at row i (other columns ignored)
static void finite_flags_f32(st_ctx *c, const std::vector<float *> &cols, uint64_t n, uint32_t *flags) {
    if (cols.empty()) {
        ST_HIP(hipMemsetD32Async(flags, 1, n, c->stream));
        return;
    }
    bool wide = cols.size() <= (size_t)WIDE_COLS;
    ColPtrs cp{};
    for (size_t i = 0; wide && i < cols.size(); ++i) {
        cp.p[i] = cols[i];
        wide = aligned16(cols[i]);
    }
    if (wide) {
        hipLaunchKernelGGL(k_finite_flags4, dim3(grid_for((n + 3) / 4, 256, 8192)), dim3(256), 0, c->stream, cp,
                           (int)cols.size(), n, flags);
    } else {
        float *const *dcols = upload_ptrs(c, "filter.cols", cols);
        hipLaunchKernelGGL(k_finite_flags, dim3(grid_for(n, 256, 8192)), dim3(256), 0, c->stream, dcols,
                           (int)cols.size(), n, flags);
    }
    ST_LAUNCH_CHECK();
}

uint64_t filter_finite_tdev(st_ctx *c, const st_ttable *t, uint32_t *out_idx) {
    const uint64_t n = t->n;
    if (n == 0) return 0;
    auto *flags = wsT<uint32_t>(c, "filter.flags", n);
    std::vector<float *> f32;
    std::vector<double *> f64;
    for (int i = 0; i < t->ncol; ++i) {
        if (t->types[i] == ST_PLY_FLOAT) f32.push_back(static_cast<float *>(t->cols[i]));
        if (t->types[i] == ST_PLY_DOUBLE) f64.push_back(static_cast<double *>(t->cols[i]));
    }
    finite_flags_f32(c, f32, n, flags);
    if (!f64.empty()) {
        double *const *d = upload_ptrs(c, "filter.cols64", f64);
        hipLaunchKernelGGL(k_finite_and_f64, dim3(grid_for(n, 256, 8192)), dim3(256), 0, c->stream, d, (int)f64.size(),
                           n, flags);
        ST_LAUNCH_CHECK();
    }
    return compact_flags_dev(c, flags, n, out_idx);
}

uint64_t compact_flags_dev(st_ctx *c, const uint32_t *flags, uint64_t n, uint32_t *out_idx) {
    if (n == 0) return 0;
    auto *pos = wsT<uint32_t>(c, "filter.pos", n + 1);
    scan_u32(c, flags, pos, n, pos + n);
    hipLaunchKernelGGL(k_compact, dim3(grid_for(n, 256, 8192)), dim3(256), 0, c->stream, flags, pos, n, out_idx);
    ST_LAUNCH_CHECK();
    auto *h = static_cast<uint32_t *>(pinned(c, 16));
    ST_HIP(hipMemcpyAsync(h, pos + n, sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
    ST_HIP(hipStreamSynchronize(c->stream));
    return h[0];
}

// filterByValue (process.ts:97-109): row[columnName] <cmp> value on the column's value as a JS
// number (every column type converts to f64 exactly).  NaN compares false except !==; a
// missing column reads undefined (NaN); an unknown comparator keeps every row (:108)
uint64_t filter_value_tdev(st_ctx *c, const st_ttable *t, const char *column, int32_t cmp, double value,
                           uint32_t *out_idx) {
    const uint64_t n = t->n;
    if (n == 0) return 0;
    auto *flags = wsT<uint32_t>(c, "filter.flags", n);
    int col = -1;
    for (int i = 0; i < t->ncol && col < 0; ++i)
        if (column && std::strcmp(t->names[i], column) == 0) col = i;
    const unsigned g = grid_for(n, 256, 8192);
    if (cmp < ST_CMP_LT || cmp > ST_CMP_NEQ) {
        ST_HIP(hipMemsetD32Async(flags, 1, n, c->stream));
    } else if (col < 0) {
        ST_HIP(hipMemsetD32Async(flags, cmp == ST_CMP_NEQ ? 1 : 0, n, c->stream));
    } else {
        void *p = t->cols[col];
        switch (t->types[col]) {
            case ST_PLY_CHAR: hipLaunchKernelGGL(k_cmp_flags<int8_t>, dim3(g), dim3(256), 0, c->stream, (const int8_t *)p, n, cmp, value, flags); break;
            case ST_PLY_UCHAR: hipLaunchKernelGGL(k_cmp_flags<uint8_t>, dim3(g), dim3(256), 0, c->stream, (const uint8_t *)p, n, cmp, value, flags); break;
            case ST_PLY_SHORT: hipLaunchKernelGGL(k_cmp_flags<int16_t>, dim3(g), dim3(256), 0, c->stream, (const int16_t *)p, n, cmp, value, flags); break;
            case ST_PLY_USHORT: hipLaunchKernelGGL(k_cmp_flags<uint16_t>, dim3(g), dim3(256), 0, c->stream, (const uint16_t *)p, n, cmp, value, flags); break;
            case ST_PLY_INT: hipLaunchKernelGGL(k_cmp_flags<int32_t>, dim3(g), dim3(256), 0, c->stream, (const int32_t *)p, n, cmp, value, flags); break;
            case ST_PLY_UINT: hipLaunchKernelGGL(k_cmp_flags<uint32_t>, dim3(g), dim3(256), 0, c->stream, (const uint32_t *)p, n, cmp, value, flags); break;
            case ST_PLY_FLOAT: hipLaunchKernelGGL(k_cmp_flags<float>, dim3(g), dim3(256), 0, c->stream, (const float *)p, n, cmp, value, flags); break;
            case ST_PLY_DOUBLE: hipLaunchKernelGGL(k_cmp_flags<double>, dim3(g), dim3(256), 0, c->stream, (const double *)p, n, cmp, value, flags); break;
            default: throw Error(ST_ERR_ARG, "filterByValue: bad column type");
        }
        ST_LAUNCH_CHECK();
    }
    return compact_flags_dev(c, flags, n, out_idx);
}

template <typename T>
static void gather_sized(st_ctx *c, const char *slot, const std::vector<void *> &s, const std::vector<void *> &d,
                         const uint32_t *idx, uint64_t m) {
    if (s.empty()) return;
    std::vector<T *> sp, dp;
    for (size_t i = 0; i < s.size(); ++i) {
        sp.push_back(static_cast<T *>(s[i]));
        dp.push_back(static_cast<T *>(d[i]));
    }
    T *const *ds = upload_ptrs(c, std::string(slot) + ".s", sp);
    T *const *dd = upload_ptrs(c, std::string(slot) + ".d", dp);
    hipLaunchKernelGGL(k_gather_t<T>, dim3(grid_for(m, 256, 8192)), dim3(256), 0, c->stream, ds, dd, (int)s.size(),
                       idx, m);
    ST_LAUNCH_CHECK();
}

void permute_rows_tdev(st_ctx *c, const st_ttable *src, const uint32_t *idx, uint64_t m, const st_ttable *dst) {
    if (m == 0 || src->ncol == 0) return;
    std::vector<void *> s[4], d[4];  // by element size 1, 2, 4, 8
    for (int i = 0; i < src->ncol; ++i) {
        const int sz = type_size(src->types[i]);
        const int b = sz == 1 ? 0 : sz == 2 ? 1 : sz == 4 ? 2 : 3;
        s[b].push_back(src->cols[i]);
        d[b].push_back(dst->cols[i]);
    }
    // 4-byte columns: the wide kernel in groups of up to WIDE_COLS columns
    for (size_t g0 = 0; g0 < s[2].size(); g0 += WIDE_COLS) {
        const size_t g1 = std::min(s[2].size(), g0 + (size_t)WIDE_COLS);
        bool wide = aligned16(idx);
        ColPtrs sp{}, dp{};
        for (size_t i = g0; i < g1; ++i) {
            sp.p[i - g0] = static_cast<const float *>(s[2][i]);
            dp.p[i - g0] = static_cast<const float *>(d[2][i]);
            wide = wide && aligned16(d[2][i]);
        }
        if (wide) {
            hipLaunchKernelGGL(k_gather_cols4, dim3(grid_for((m + 3) / 4, 256, 8192)), dim3(256), 0, c->stream, sp, dp,
                               (int)(g1 - g0), idx, m);
            ST_LAUNCH_CHECK();
        } else {
            std::vector<void *> ss(s[2].begin() + g0, s[2].begin() + g1), dd(d[2].begin() + g0, d[2].begin() + g1);
            gather_sized<float>(c, "permute.f4", ss, dd, idx, m);
        }
    }
    gather_sized<uint8_t>(c, "permute.b1", s[0], d[0], idx, m);
    gather_sized<uint16_t>(c, "permute.b2", s[1], d[1], idx, m);
    gather_sized<uint64_t>(c, "permute.b8", s[3], d[3], idx, m);
}

static bool same_name(const char *a, const char *b) { return std::strcmp(a, b) == 0; }

// combine's column list: (table, column) of each result column in the reference's order
// (the first table's columns, then each later table's columns without a (name, type) match)
int combine_layout(const st_ttable *const *srcs, int nsrc, int32_t *col_table, int32_t *col_index) {
    int nout = 0;
    std::vector<std::pair<int, int>> out;
    for (int t = 0; t < nsrc; ++t) {
        for (int j = 0; j < srcs[t]->ncol; ++j) {
            bool found = false;
            for (auto &o : out)
                found = found || (same_name(srcs[o.first]->names[o.second], srcs[t]->names[j]) &&
                                  srcs[o.first]->types[o.second] == srcs[t]->types[j]);
            // the first table's columns are copied as they are (index.ts:175), duplicates included
            if (!found || t == 0) out.emplace_back(t, j);
        }
    }
    for (auto &o : out) {
        if (col_table) col_table[nout] = o.first;
        if (col_index) col_index[nout] = o.second;
        ++nout;
    }
    return nout;
}

// dst: the combine_layout columns with sum(n) rows.  The result is zero-filled, then every
// source column is copied to the FIRST result column of its (name, type) at the table's row
// offset (targetColumn.data.set(column.data, rowOffset), index.ts:197-205)
void combine_tdev(st_ctx *c, const st_ttable *const *srcs, int nsrc, const st_ttable *dst) {
    uint64_t total = 0;
    for (int i = 0; i < nsrc; ++i) total += srcs[i]->n;
    ST_REQUIRE(total == dst->n, ST_ERR_ARG, "combine: dst rows != sum of src rows");
    for (int j = 0; j < dst->ncol; ++j)
        if (total) ST_HIP(hipMemsetAsync(dst->cols[j], 0, total * type_size(dst->types[j]), c->stream));
    uint64_t off = 0;
    for (int t = 0; t < nsrc; ++t) {
        const st_ttable *s = srcs[t];
        for (int j = 0; j < s->ncol && s->n; ++j) {
            int target = -1;
            for (int k = 0; k < dst->ncol && target < 0; ++k)
                if (same_name(dst->names[k], s->names[j]) && dst->types[k] == s->types[j]) target = k;
            ST_REQUIRE(target >= 0, ST_ERR_ARG, std::string("combine: dst lacks column ") + s->names[j]);
            const int sz = type_size(s->types[j]);
            ST_HIP(hipMemcpyAsync(static_cast<char *>(dst->cols[target]) + off * sz, s->cols[j], s->n * sz,
                                  hipMemcpyDeviceToDevice, c->stream));
        }
        off += s->n;
    }
}

// float32-only forms (st_table): the typed ones with every column ST_PLY_FLOAT
struct F32View {
    std::vector<int32_t> types;
    std::vector<void *> cols;
    st_ttable t{};
    explicit F32View(const st_table *s) : types(s->ncol, ST_PLY_FLOAT), cols(s->cols, s->cols + s->ncol) {
        t.n = s->n;
        t.ncol = s->ncol;
        t.names = s->names;
        t.types = types.data();
        t.cols = cols.data();
    }
};

uint64_t filter_finite_dev(st_ctx *c, const st_table *t, uint32_t *out_idx) {
    F32View v(t);
    return filter_finite_tdev(c, &v.t, out_idx);
}

void permute_rows_dev(st_ctx *c, const st_table *src, const uint32_t *idx, uint64_t m, const st_table *dst) {
    F32View s(src), d(dst);
    permute_rows_tdev(c, &s.t, idx, m, &d.t);
}

void concat_rows_dev(st_ctx *c, const st_table *const *srcs, int nsrc, const st_table *dst) {
    std::vector<F32View> v;
    v.reserve(nsrc);
    std::vector<const st_ttable *> p;
    for (int i = 0; i < nsrc; ++i) v.emplace_back(srcs[i]);
    for (auto &x : v) p.push_back(&x.t);
    F32View d(dst);
    combine_tdev(c, p.data(), nsrc, &d.t);
}

}  // namespace st
