// st_typed.h -- JS typed-array element semantics for the reference's eight column types.
//
// The reference reads any column through getRow (data-table.ts:63-68: the element as a JS
// number) and writes through setRow (:70-76: a TypedArray element store).  A store converts
// the number as ECMA-262 IntegerIndexedElementSet does: Float32 rounds to nearest even,
// Float64 keeps it, the integer types take ToInt32 (truncation toward zero, modulo 2^32, NaN
// and +-Infinity -> 0) cut to their width (Uint8Array is not clamped).
#pragma once

#include "st_internal.h"
#include "st_jsmath.h"

namespace st {

// element i of a column of type t (ST_PLY_*) as a JS number
__host__ __device__ inline double ta_load(const void *p, int32_t t, uint64_t i) {
    switch (t) {
        case ST_PLY_CHAR: return (double)static_cast<const int8_t *>(p)[i];
        case ST_PLY_UCHAR: return (double)static_cast<const uint8_t *>(p)[i];
        case ST_PLY_SHORT: return (double)static_cast<const int16_t *>(p)[i];
        case ST_PLY_USHORT: return (double)static_cast<const uint16_t *>(p)[i];
        case ST_PLY_INT: return (double)static_cast<const int32_t *>(p)[i];
        case ST_PLY_UINT: return (double)static_cast<const uint32_t *>(p)[i];
        case ST_PLY_FLOAT: return (double)static_cast<const float *>(p)[i];
        default: return static_cast<const double *>(p)[i];
    }
}

// element i of a column of type t := the JS number v
__host__ __device__ inline void ta_store(void *p, int32_t t, uint64_t i, double v) {
    switch (t) {
        case ST_PLY_CHAR: static_cast<int8_t *>(p)[i] = (int8_t)(uint8_t)js::to_uint32(v); break;
        case ST_PLY_UCHAR: static_cast<uint8_t *>(p)[i] = (uint8_t)js::to_uint32(v); break;
        case ST_PLY_SHORT: static_cast<int16_t *>(p)[i] = (int16_t)(uint16_t)js::to_uint32(v); break;
        case ST_PLY_USHORT: static_cast<uint16_t *>(p)[i] = (uint16_t)js::to_uint32(v); break;
        case ST_PLY_INT: static_cast<int32_t *>(p)[i] = js::to_int32(v); break;
        case ST_PLY_UINT: static_cast<uint32_t *>(p)[i] = js::to_uint32(v); break;
        case ST_PLY_FLOAT: static_cast<float *>(p)[i] = (float)v; break;
        default: static_cast<double *>(p)[i] = v; break;
    }
}

// a typed device column
struct TCol {
    void *p;
    int32_t t;
};

// column `name` of a typed table (p = nullptr if absent)
TCol tcol_or_null(const st_ttable *t, const char *name);
// the Float32Array copy of a typed device column (getRow -> Float32Array element, as the
// reference's chunk members, cluster1d data and k-means points are): the column itself when
// it is float32, else a workspace slot `slot`
const float *as_f32_dev(st_ctx *c, TCol col, uint64_t n, const std::string &slot);
// the JS numbers of a typed device column as float64 (exact for every type): workspace `slot`
const double *as_f64_dev(st_ctx *c, TCol col, uint64_t n, const std::string &slot);
// true when every one of the named columns present in t is float32
bool all_f32(const st_ttable *t, const char *const *names, int count);

}  // namespace st
