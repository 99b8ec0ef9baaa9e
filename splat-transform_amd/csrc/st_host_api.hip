// st_host_api.hip -- host-memory entry points: copy the borrowed host columns
// into HBM, run the device path, copy results back.  These mirror the
// reference seams one-for-one for callers that hold host TypedArrays (the
// N-API addon, ctypes); callers that keep tables resident use st_dev_*.
#include <cstdlib>
#include <cstring>

#include "st_internal.h"
#include "st_webp.h"

namespace st {
namespace {

struct DevTable {
    std::vector<std::string> names;
    std::vector<const char *> cnames;
    std::vector<float *> cols;
    st_table t{};
};

// upload the named subset (or all columns when `want` is empty) of a host table
DevTable upload(st_ctx *c, const st_table *h, const std::vector<std::string> &want, const std::string &tag) {
    DevTable d;
    for (int i = 0; i < h->ncol; ++i) {
        if (!want.empty()) {
            bool hit = false;
            for (auto &w : want) hit = hit || (w == h->names[i]);
            if (!hit) continue;
        }
        d.names.push_back(h->names[i]);
    }
    for (size_t i = 0; i < d.names.size(); ++i) {
        const int src = find_col(h, d.names[i].c_str());
        float *p = wsT<float>(c, tag + std::to_string(i), h->n);
        if (h->n) ST_HIP(hipMemcpyAsync(p, h->cols[src], h->n * 4, hipMemcpyHostToDevice, c->stream));
        d.cols.push_back(p);
    }
    for (auto &s : d.names) d.cnames.push_back(s.c_str());
    d.t.n = h->n;
    d.t.ncol = (int32_t)d.names.size();
    d.t.names = d.cnames.data();
    d.t.cols = d.cols.data();
    return d;
}

void download(st_ctx *c, const DevTable &d, const st_table *h) {
    for (size_t i = 0; i < d.names.size(); ++i) {
        const int dst = find_col(h, d.names[i].c_str());
        if (h->n) ST_HIP(hipMemcpyAsync(h->cols[dst], d.cols[i], h->n * 4, hipMemcpyDeviceToHost, c->stream));
    }
    ST_HIP(hipStreamSynchronize(c->stream));
}

std::vector<std::string> transform_columns() {
    std::vector<std::string> v = {"x", "y", "z", "rot_0", "rot_1", "rot_2", "rot_3", "scale_0", "scale_1", "scale_2"};
    for (int i = 0; i < 45; ++i) v.push_back("f_rest_" + std::to_string(i));
    return v;
}

template <typename T>
T *to_dev(st_ctx *c, const std::string &slot, const T *h, size_t count) {
    T *d = wsT<T>(c, slot, count);
    if (count) ST_HIP(hipMemcpyAsync(d, h, count * sizeof(T), hipMemcpyHostToDevice, c->stream));
    return d;
}

template <typename T>
void to_host(st_ctx *c, T *h, const T *d, size_t count) {
    if (count) ST_HIP(hipMemcpyAsync(h, d, count * sizeof(T), hipMemcpyDeviceToHost, c->stream));
}

}  // namespace
}  // namespace st

using namespace st;

template <typename F>
static int guarded_h(F &&f) {
    try {
        f();
        return ST_OK;
    } catch (const st::Error &e) {
        set_last_error(e.what());
        return e.code;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        return ST_ERR_INTERNAL;
    }
}

#define ST_ARGH(cond, msg) ST_REQUIRE(cond, ST_ERR_ARG, msg)

extern "C" {

int st_transform(st_ctx *c, const st_table *t, const st_transform_params *p) {
    return guarded_h([&] {
        ST_ARGH(c && t && p, "NULL argument");
        use_device(c);
        DevTable d = upload(c, t, transform_columns(), "h.t");
        transform_dev(c, &d.t, p);
        download(c, d, t);
    });
}

int st_filter_finite(st_ctx *c, const st_table *t, uint32_t *out_idx, uint64_t *out_n) {
    return guarded_h([&] {
        ST_ARGH(c && t && out_idx && out_n, "NULL argument");
        use_device(c);
        DevTable d = upload(c, t, {}, "h.f");
        auto *didx = wsT<uint32_t>(c, "h.fidx", t->n);
        const uint64_t m = filter_finite_dev(c, &d.t, didx);
        to_host(c, out_idx, didx, m);
        ST_HIP(hipStreamSynchronize(c->stream));
        *out_n = m;
    });
}

int st_filter_nan(st_ctx *c, const st_ttable *src, const st_ttable *dst, uint64_t *out_m) {
    return guarded_h([&] {
        ST_ARGH(c && src && dst && out_m, "NULL argument");
        ST_ARGH(src->ncol == dst->ncol && dst->n >= src->n, "filter_nan: dst needs src's columns and n rows");
        use_device(c);
        const uint64_t n = src->n;
        std::vector<void *> dcols(src->ncol), ocols(src->ncol);
        for (int i = 0; i < src->ncol; ++i) {
            const int sz = type_size(src->types[i]);
            ST_ARGH(sz > 0 && dst->types[i] == src->types[i], "filter_nan: bad or mismatched column type");
            dcols[i] = ws(c, "h.fn" + std::to_string(i), n * sz + 16);
            if (n) ST_HIP(hipMemcpyAsync(dcols[i], src->cols[i], n * sz, hipMemcpyHostToDevice, c->stream));
        }
        st_ttable d = *src;
        d.cols = dcols.data();
        auto *didx = wsT<uint32_t>(c, "h.fnidx", n);
        const uint64_t m = filter_finite_tdev(c, &d, didx);
        for (int i = 0; i < src->ncol; ++i) ocols[i] = ws(c, "h.fno" + std::to_string(i), m * type_size(src->types[i]) + 16);
        st_ttable o = d;
        o.n = m;
        o.cols = ocols.data();
        permute_rows_tdev(c, &d, didx, m, &o);
        for (int i = 0; i < src->ncol; ++i)
            if (m) ST_HIP(hipMemcpyAsync(dst->cols[i], ocols[i], m * type_size(src->types[i]), hipMemcpyDeviceToHost,
                                         c->stream));
        ST_HIP(hipStreamSynchronize(c->stream));
        *out_m = m;
    });
}

int st_morton_order(st_ctx *c, const float *x, const float *y, const float *z, uint32_t *idx, uint64_t n) {
    return guarded_h([&] {
        ST_ARGH(c && ((x && y && z && idx) || n == 0), "NULL argument");
        if (n == 0) return;
        use_device(c);
        float *dx = to_dev(c, "h.mx", x, n), *dy = to_dev(c, "h.my", y, n), *dz = to_dev(c, "h.mz", z, n);
        uint32_t *di = to_dev(c, "h.mi", idx, n);
        morton_order_dev(c, dx, dy, dz, di, n);
        to_host(c, idx, di, n);
        ST_HIP(hipStreamSynchronize(c->stream));
    });
}

int st_pack_compressed(st_ctx *c, const st_table *t, const uint32_t *order, float *chunk, uint32_t *vertex,
                       uint8_t *sh) {
    return guarded_h([&] {
        ST_ARGH(c && t && ((order && chunk && vertex) || t->n == 0), "NULL argument");
        if (t->n == 0) return;
        use_device(c);
        DevTable d = upload(c, t, {}, "h.c");
        const uint64_t n = t->n, nch = (n + 255) / 256;
        const int nsh = 3 * sh_coeffs_of(t);
        uint32_t *dord = to_dev(c, "h.cord", order, n);
        auto *dchunk = wsT<float>(c, "h.cchunk", nch * 18);
        auto *dvert = wsT<uint32_t>(c, "h.cvert", n * 4);
        auto *dsh = wsT<uint8_t>(c, "h.csh", n * (uint64_t)nsh + 1);
        pack_compressed_dev(c, &d.t, dord, dchunk, dvert, dsh);
        to_host(c, chunk, dchunk, nch * 18);
        to_host(c, vertex, dvert, n * 4);
        if (nsh) to_host(c, sh, dsh, n * (uint64_t)nsh);
        ST_HIP(hipStreamSynchronize(c->stream));
    });
}

int st_kmeans(st_ctx *c, const float *const *cols, int32_t d, uint64_t n, int32_t k, int32_t iters,
              const double *draws, uint64_t ndraws, uint64_t *used, float *centroids, uint32_t *labels) {
    return guarded_h([&] {
        ST_ARGH(c && cols && d > 0 && k > 0 && centroids && labels, "bad argument");
        use_device(c);
        std::vector<const float *> dc(d);
        for (int j = 0; j < d; ++j) dc[j] = to_dev(c, "h.k" + std::to_string(j), cols[j], n);
        const uint64_t kk = n < (uint64_t)k ? n : (uint64_t)k;
        auto *dcen = wsT<float>(c, "h.kcen", (size_t)d * (k > (int)kk ? k : kk));
        auto *dlab = wsT<uint32_t>(c, "h.klab", n);
        const uint64_t u = kmeans_dev(c, dc.data(), d, n, k, iters, draws, ndraws, dcen, dlab);
        to_host(c, centroids, dcen, (size_t)d * kk);
        to_host(c, labels, dlab, n);
        ST_HIP(hipStreamSynchronize(c->stream));
        if (used) *used = u;
    });
}

int st_cluster1d(st_ctx *c, const float *const *cols, int32_t ncols, uint64_t n, int32_t iters, const double *draws,
                 uint64_t ndraws, uint64_t *used, float *centroids256, uint8_t *labels) {
    return guarded_h([&] {
        ST_ARGH(c && cols && ncols > 0 && centroids256 && labels, "bad argument");
        use_device(c);
        std::vector<const float *> dc(ncols);
        for (int j = 0; j < ncols; ++j) dc[j] = to_dev(c, "h.1d" + std::to_string(j), cols[j], n);
        auto *dcen = wsT<float>(c, "h.1dcen", 256);
        auto *dlab = wsT<uint8_t>(c, "h.1dlab", n * (uint64_t)ncols);
        const uint64_t u = cluster1d_dev(c, dc.data(), ncols, n, iters, draws, ndraws, dcen, dlab);
        to_host(c, centroids256, dcen, 256);
        to_host(c, labels, dlab, n * (uint64_t)ncols);
        ST_HIP(hipStreamSynchronize(c->stream));
        if (used) *used = u;
    });
}

int st_sog(st_ctx *c, const st_table *t, int32_t iters, const double *draws, uint64_t ndraws, uint64_t *used,
           st_sog_meta *meta, const st_sog_textures *out) {
    if (int rc = apply_env_devices()) return rc;
    if (st_group *g = default_group()) return st_group_sog(g, &t, 1, nullptr, iters, draws, ndraws, used, meta, out);
    return guarded_h([&] {
        ST_ARGH(c && t && meta && out, "NULL argument");
        use_device(c);
        DevTable d = upload(c, t, {}, "h.s");
        const int C = sh_coeffs_of(t);
        int32_t W, H, pal, cw, chh;
        ST_REQUIRE(st_sog_geometry(t->n, C, &W, &H, &pal, &cw, &chh) == ST_OK, ST_ERR_ARG, "sog: empty table");
        const uint64_t tex = (uint64_t)W * H * 4;
        st_sog_textures dt{};
        dt.means_l = wsT<uint8_t>(c, "h.s.ml", tex);
        dt.means_u = wsT<uint8_t>(c, "h.s.mu", tex);
        dt.quats = wsT<uint8_t>(c, "h.s.q", tex);
        dt.scales = wsT<uint8_t>(c, "h.s.sc", tex);
        dt.sh0 = wsT<uint8_t>(c, "h.s.sh0", tex);
        if (C) {
            dt.shn_labels = wsT<uint8_t>(c, "h.s.shl", tex);
            dt.shn_centroids = wsT<uint8_t>(c, "h.s.shc", (uint64_t)cw * chh * 4);
        }
        const uint64_t u = sog_dev(c, &d.t, iters, draws, ndraws, meta, &dt);
        to_host(c, out->means_l, dt.means_l, tex);
        to_host(c, out->means_u, dt.means_u, tex);
        to_host(c, out->quats, dt.quats, tex);
        to_host(c, out->scales, dt.scales, tex);
        to_host(c, out->sh0, dt.sh0, tex);
        if (C) {
            ST_ARGH(out->shn_labels && out->shn_centroids, "sog: shN outputs are NULL");
            to_host(c, out->shn_labels, dt.shn_labels, tex);
            to_host(c, out->shn_centroids, dt.shn_centroids, (uint64_t)cw * chh * 4);
        }
        ST_HIP(hipStreamSynchronize(c->stream));
        if (used) *used = u;
    });
}

// writeSog to a .sog bundle (write-sog.ts:110-370 with the ZipWriter of :112-114):
// the archive bytes, malloc'd (st_free)
int st_sog_bundle(st_ctx *c, const st_table *t, int32_t iters, const double *draws, uint64_t ndraws, uint64_t *used,
                  uint16_t dos_time, uint16_t dos_date, uint8_t **out, uint64_t *out_size) {
    if (int rc = apply_env_devices()) return rc;
    if (st_group *g = default_group())
        return st_group_sog_bundle(g, &t, 1, nullptr, iters, draws, ndraws, used, dos_time, dos_date, out, out_size);
    return guarded_h([&] {
        ST_ARGH(c && t && out && out_size, "NULL argument");
        use_device(c);
        DevTable d = upload(c, t, {}, "h.s");
        const int C = sh_coeffs_of(t);
        int32_t W, H, pal, cw, chh;
        ST_REQUIRE(st_sog_geometry(t->n, C, &W, &H, &pal, &cw, &chh) == ST_OK, ST_ERR_ARG, "sog: empty table");
        const uint64_t tex = (uint64_t)W * H * 4;
        st_sog_textures dt{};
        dt.means_l = wsT<uint8_t>(c, "h.s.ml", tex);
        dt.means_u = wsT<uint8_t>(c, "h.s.mu", tex);
        dt.quats = wsT<uint8_t>(c, "h.s.q", tex);
        dt.scales = wsT<uint8_t>(c, "h.s.sc", tex);
        dt.sh0 = wsT<uint8_t>(c, "h.s.sh0", tex);
        if (C) {
            dt.shn_labels = wsT<uint8_t>(c, "h.s.shl", tex);
            dt.shn_centroids = wsT<uint8_t>(c, "h.s.shc", (uint64_t)cw * chh * 4);
        }
        st_sog_meta meta{};
        const uint64_t u = sog_dev(c, &d.t, iters, draws, ndraws, &meta, &dt);
        const uint8_t *view;
        uint64_t nb;
        sog_bundle_dev(c, meta, t->n, dt, dos_time, dos_date, &view, &nb);
        uint8_t *buf = (uint8_t *)std::malloc(nb);
        ST_REQUIRE(buf, ST_ERR_NOMEM, "sog bundle: host allocation failed");
        std::memcpy(buf, view, nb);
        *out = buf;
        *out_size = nb;
        if (used) *used = u;
    });
}

}  // extern "C"
