// st_typed.hip -- typed device columns as the reference's number views (st_typed.h).
#include <cstring>

#include "st_typed.h"

namespace st {
namespace {

__global__ __launch_bounds__(256) void k_to_f32(const void *__restrict__ src, int32_t t, uint64_t n,
                                                float *__restrict__ dst) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        dst[i] = (float)ta_load(src, t, i);
}

__global__ __launch_bounds__(256) void k_to_f64(const void *__restrict__ src, int32_t t, uint64_t n,
                                                double *__restrict__ dst) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        dst[i] = ta_load(src, t, i);
}

}  // namespace

TCol tcol_or_null(const st_ttable *t, const char *name) {
    for (int i = 0; i < t->ncol; ++i)
        if (std::strcmp(t->names[i], name) == 0) return TCol{t->cols[i], t->types[i]};
    return TCol{nullptr, 0};
}

bool all_f32(const st_ttable *t, const char *const *names, int count) {
    for (int j = 0; j < count; ++j) {
        const TCol c = tcol_or_null(t, names[j]);
        if (c.p && c.t != ST_PLY_FLOAT) return false;
    }
    return true;
}

const float *as_f32_dev(st_ctx *c, TCol col, uint64_t n, const std::string &slot) {
    if (col.t == ST_PLY_FLOAT) return static_cast<const float *>(col.p);
    auto *d = wsT<float>(c, slot, n);
    if (n) {
        hipLaunchKernelGGL(k_to_f32, dim3(grid_for(n, 256, 8192)), dim3(256), 0, c->stream, col.p, col.t, n, d);
        ST_LAUNCH_CHECK();
    }
    return d;
}

const double *as_f64_dev(st_ctx *c, TCol col, uint64_t n, const std::string &slot) {
    auto *d = wsT<double>(c, slot, n);
    if (n) {
        hipLaunchKernelGGL(k_to_f64, dim3(grid_for(n, 256, 8192)), dim3(256), 0, c->stream, col.p, col.t, n, d);
        ST_LAUNCH_CHECK();
    }
    return d;
}

}  // namespace st
