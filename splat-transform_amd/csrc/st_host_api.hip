// st_host_api.hip -- host-memory entry points: copy the borrowed host columns
// into HBM, run the device path, copy results back.  These mirror the
// reference seams one-for-one for callers that hold host TypedArrays (the
// N-API addon, ctypes); callers that keep tables resident use st_dev_*.
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>

#include <unistd.h>
#include <cerrno>
#include "st_internal.h"
#include "st_webp.h"

namespace st {
namespace {

struct DevTable {
    std::vector<std::string> names;
    std::vector<const char *> cnames;
    std::vector<float *> cols;
    st_table t{};
    uint64_t resident = 0;  // columns read where they already were in HBM (resident_table)
};

// host <-> device transfers of one call, moved together through the staged copies
struct Batch {
    st_ctx *c;
    std::vector<HostXfer> v;
    template <typename T>
    void add(const T *host, T *dev, size_t count) {
        v.push_back(HostXfer{const_cast<T *>(host), dev, count * sizeof(T)});
    }
    template <typename T>
    void add_d2h(T *host, const T *dev, size_t count) {
        v.push_back(HostXfer{host, const_cast<T *>(dev), count * sizeof(T)});
    }
    void h2d() {
        staged_h2d(c, v);
        v.clear();
    }
    void d2h() {
        staged_d2h(c, v);
        v.clear();
    }
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
    Batch up{c};
    for (size_t i = 0; i < d.names.size(); ++i) {
        const int src = find_col(h, d.names[i].c_str());
        float *p = wsT<float>(c, tag + std::to_string(i), h->n);
        up.add(h->cols[src], p, h->n);
        d.cols.push_back(p);
    }
    up.h2d();
    for (auto &s : d.names) d.cnames.push_back(s.c_str());
    d.t.n = h->n;
    d.t.ncol = (int32_t)d.names.size();
    d.t.names = d.cnames.data();
    d.t.cols = d.cols.data();
    return d;
}

void download(st_ctx *c, const DevTable &d, const st_table *h) {
    Batch down{c};
    for (size_t i = 0; i < d.names.size(); ++i) {
        const int dst = find_col(h, d.names[i].c_str());
        down.add_d2h(h->cols[dst], d.cols[i], h->n);
    }
    down.d2h();
}

// the columns writeSog reads (write-sog.ts:110-370): the other columns of a PLY (normals, extra
// properties) are not uploaded
std::vector<std::string> sog_columns() {
    std::vector<std::string> v = {"x", "y", "z", "scale_0", "scale_1", "scale_2", "f_dc_0",
                                  "f_dc_1", "f_dc_2", "opacity", "rot_0", "rot_1", "rot_2", "rot_3"};
    for (int i = 0; i < 45; ++i) v.push_back("f_rest_" + std::to_string(i));
    return v;
}

std::vector<std::string> transform_columns() {
    std::vector<std::string> v = {"x", "y", "z", "rot_0", "rot_1", "rot_2", "rot_3", "scale_0", "scale_1", "scale_2"};
    for (int i = 0; i < 45; ++i) v.push_back("f_rest_" + std::to_string(i));
    return v;
}

// ---- writeSog host forms on resident columns (st_ctx::HostMirror) ---------------------------
// A column writeSog reads that is resident in HBM is not uploaded:
//  * a lazy column (st_ply_read_resident: its host memory was never filled) is read on the
//    device as it is -- its values exist nowhere else;
//  * a mirrored column (st_ply_read filled it and a host twin) is read on the device while host
//    threads compare the caller's column with the twin byte for byte (memcmp, ~4.7 GB read at
//    10M splats, beside the step).  Nothing leaves the device (no file write, no host output) until
//    the compare has said "equal"; a changed byte raises spec_abort (the SH k-means stops at its
//    next iteration), the call waits for its queued work and runs again with those columns
//    uploaded.
// Every other column is uploaded.
struct Spec {
    st_ctx *c;
    std::atomic<bool> abort{false};
    std::vector<std::thread> th;
    std::mutex mu;  // verdict() is called from the call's thread and from sog_file_dev's writer
    bool joined = false;
    explicit Spec(st_ctx *ctx) : c(ctx) {}
    bool verdict() {
        std::lock_guard<std::mutex> lk(mu);
        if (!joined) {
            for (auto &t : th) t.join();
            joined = true;
        }
        return !abort.load();
    }
    ~Spec() {
        verdict();
        c->spec_abort = nullptr;
        c->spec_verdict = nullptr;
    }
};

// the wanted float columns of h on the device: resident ones as they are (mirrored ones under sp's
// compare; without sp they are uploaded like the rest), the others uploaded into `tag` slots.
// False (nothing done) when none is resident.  d.resident counts the columns not uploaded.
bool resident_table(st_ctx *c, const st_table *h, const std::vector<std::string> &want, DevTable &d, Spec *sp,
                    const std::string &tag) {
    const char *mo = getenv("ST_HOST_MIRROR");
    const bool compare_ok = sp && !(mo && std::strcmp(mo, "0") == 0);
    std::lock_guard<std::mutex> lk(c->mirror_mu);
    if (c->mirrors.empty() || !h->n) return false;
    std::vector<int> src;
    std::vector<st_ctx::HostMirror> ms;  // copies: the list may change once the lock is released
    bool any = false;
    for (int i = 0; i < h->ncol; ++i) {
        bool hit = want.empty();
        for (auto &w : want) hit = hit || (w == h->names[i]);
        if (!hit) continue;
        st_ctx::HostMirror m{};
        for (const auto &x : c->mirrors)
            if (x.host == h->cols[i] && x.bytes == h->n * sizeof(float) && (x.lazy || compare_ok)) m = x;
        any = any || m.host;
        src.push_back(i);
        ms.push_back(m);
    }
    if (!any) return false;
    // a column read from host memory that lies inside a lazy one (a view of it) is copied down first
    {
        std::vector<HostXfer> down;
        std::vector<const void *> gone;
        for (size_t j = 0; j < src.size(); ++j) {
            if (ms[j].host) continue;
            const char *a = static_cast<const char *>(static_cast<const void *>(h->cols[src[j]]));
            for (const auto &x : c->mirrors) {
                const char *b = static_cast<const char *>(x.host);
                if (x.lazy && a < b + x.bytes && b < a + h->n * sizeof(float)) {
                    down.push_back(HostXfer{const_cast<void *>(x.host), const_cast<void *>(x.dev), (size_t)x.bytes});
                    gone.push_back(x.host);
                }
            }
        }
        if (!down.empty()) {
            staged_d2h_raw(c, down);
            drop_mirrors_locked(c, [&](const st_ctx::HostMirror &x) {
                return std::find(gone.begin(), gone.end(), x.host) != gone.end();
            });
        }
    }
    Batch up{c};
    std::vector<std::pair<const char *, const char *>> blocks;  // the compare: 1 MiB blocks
    std::vector<uint64_t> lens;
    constexpr uint64_t BLK = 1ull << 20;
    for (size_t j = 0; j < src.size(); ++j) {
        d.names.push_back(h->names[src[j]]);
        const auto &m = ms[j];
        if (!m.host) {
            float *p = wsT<float>(c, tag + std::to_string(j), h->n);
            up.v.push_back(HostXfer{static_cast<void *>(h->cols[src[j]]), p, h->n * sizeof(float)});
            d.cols.push_back(p);
            continue;
        }
        d.cols.push_back(static_cast<float *>(const_cast<void *>(m.dev)));
        ++d.resident;
        if (!m.lazy)
            for (uint64_t o = 0; o < m.bytes; o += BLK) {
                blocks.emplace_back(static_cast<const char *>(m.host) + o, static_cast<const char *>(m.shadow) + o);
                lens.push_back(std::min(BLK, m.bytes - o));
            }
    }
    if (!up.v.empty()) {
        std::vector<HostXfer> v;
        v.swap(up.v);
        // (the lock is held: staged_h2d's own bookkeeping would take it again, and these sources are
        // not lazy -- the lazy ones are read on the device)
        staged_h2d_raw(c, v);
    }
    for (auto &s : d.names) d.cnames.push_back(s.c_str());
    d.t.n = h->n;
    d.t.ncol = (int32_t)d.names.size();
    d.t.names = d.cnames.data();
    d.t.cols = d.cols.data();
    if (blocks.empty()) return true;
    const int nt = std::max(1, std::min(16, getenv("ST_MIRROR_THREADS") ? atoi(getenv("ST_MIRROR_THREADS")) : 8));
    auto shared = std::make_shared<std::pair<decltype(blocks), decltype(lens)>>(std::move(blocks), std::move(lens));
    for (int t = 0; t < nt; ++t)
        sp->th.emplace_back([sp, shared, t, nt] {
            const auto &bl = shared->first;
            const auto &ln = shared->second;
            for (size_t b = (size_t)t; b < bl.size(); b += (size_t)nt) {
                if (sp->abort.load(std::memory_order_relaxed)) return;
                if (std::memcmp(bl[b].first, bl[b].second, ln[b]) != 0) {
                    sp->abort.store(true);
                    return;
                }
            }
        });
    c->spec_abort = &sp->abort;
    c->spec_verdict = [sp] { return sp->verdict(); };
    return true;
}

// waits for everything queued on the context's streams (an abandoned speculative run's work)
void drain_ctx(st_ctx *c) {
    for (st_ctx *x : {c, c->aux}) {
        if (!x) continue;
        (void)hipStreamSynchronize(x->stream);
        if (x->side) (void)hipStreamSynchronize(x->side);
    }
}

// body(dev_table) on the resident columns when there are any (spec_gate inside body before any
// output leaves the device), else -- or when a mirrored column changed -- with those uploaded
template <typename F>
void run_host_sog(st_ctx *c, const st_table *t, const std::vector<std::string> &want, const std::string &tag, F &&body) {
    c->last_reuse_cols = c->last_reuse_bytes = 0;
    {
        DevTable d;
        Spec sp(c);
        if (resident_table(c, t, want, d, &sp, tag)) {
            std::exception_ptr err;
            try {
                body(&d.t);
            } catch (...) {
                err = std::current_exception();
            }
            if (sp.verdict()) {
                if (err) std::rethrow_exception(err);
                c->last_reuse_cols = d.resident;
                c->last_reuse_bytes = d.resident * t->n * sizeof(float);
                return;
            }
            drain_ctx(c);
        }
    }
    {
        DevTable d;
        if (resident_table(c, t, want, d, nullptr, tag)) {  // lazy columns still from HBM
            body(&d.t);
            c->last_reuse_cols = d.resident;
            c->last_reuse_bytes = d.resident * t->n * sizeof(float);
            return;
        }
    }
    DevTable d = upload(c, t, want, tag);
    body(&d.t);
}

// a workspace slot that receives `count` host elements with the batch's next h2d()
template <typename T>
T *to_dev(Batch &b, const std::string &slot, const T *h, size_t count) {
    T *d = wsT<T>(b.c, slot, count);
    b.add(h, d, count);
    return d;
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

// transform() on a typed host table, in place: the transformed columns (x y z rot_* scale_*
// f_rest_*, any type) go up, through the typed kernel, and back
int st_transform_t(st_ctx *c, const st_ttable *t, const st_transform_params *p) {
    return guarded_h([&] {
        ST_ARGH(c && t && p && (t->ncol == 0 || (t->names && t->types && t->cols)), "NULL argument");
        use_device(c);
        const auto want = transform_columns();
        std::vector<const char *> names;
        std::vector<int32_t> types;
        std::vector<void *> dcols;
        std::vector<int> src;
        Batch b{c};
        for (int i = 0; i < t->ncol; ++i) {
            bool hit = false;
            for (auto &w : want) hit = hit || (w == t->names[i]);
            if (!hit) continue;
            const int sz = type_size(t->types[i]);
            ST_ARGH(sz > 0 && (t->cols[i] || t->n == 0), "transform: bad column");
            void *d = ws(c, "h.tt" + std::to_string(i), t->n * sz + 16);
            b.add(static_cast<const char *>(t->cols[i]), static_cast<char *>(d), t->n * sz);
            names.push_back(t->names[i]);
            types.push_back(t->types[i]);
            dcols.push_back(d);
            src.push_back(i);
        }
        b.h2d();
        const st_ttable d{t->n, (int32_t)names.size(), names.data(), types.data(), dcols.data()};
        transform_tdev(c, &d, p);
        for (size_t j = 0; j < src.size(); ++j)
            b.add_d2h(static_cast<char *>(t->cols[src[j]]), static_cast<const char *>(dcols[j]),
                      t->n * type_size(types[j]));
        b.d2h();
    });
}

// generateOrdering of x / y / z columns of any types (ST_PLY_*)
int st_morton_order_t(st_ctx *c, const void *const xyz[3], const int32_t types[3], uint32_t *idx, uint64_t n) {
    return guarded_h([&] {
        ST_ARGH(c && xyz && types && ((xyz[0] && xyz[1] && xyz[2] && idx) || n == 0), "NULL argument");
        if (n == 0) return;
        use_device(c);
        Batch b{c};
        const void *d[3];
        for (int a = 0; a < 3; ++a) {
            const int sz = type_size(types[a]);
            ST_ARGH(sz > 0, "morton: bad column type");
            char *p = static_cast<char *>(ws(c, "h.mt" + std::to_string(a), n * sz + 16));
            b.add(static_cast<const char *>(xyz[a]), p, n * sz);
            d[a] = p;
        }
        uint32_t *di = to_dev(b, "h.mi", idx, n);
        b.h2d();
        morton_order_tdev(c, d, types, di, n);
        b.add_d2h(idx, di, n);
        b.d2h();
    });
}

int st_filter_finite(st_ctx *c, const st_table *t, uint32_t *out_idx, uint64_t *out_n) {
    return guarded_h([&] {
        ST_ARGH(c && t && out_idx && out_n, "NULL argument");
        use_device(c);
        DevTable d = upload(c, t, {}, "h.f");
        auto *didx = wsT<uint32_t>(c, "h.fidx", t->n);
        const uint64_t m = filter_finite_dev(c, &d.t, didx);
        Batch b{c};
        b.add_d2h(out_idx, didx, m);
        b.d2h();
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
        Batch b{c};
        for (int i = 0; i < src->ncol; ++i) {
            const int sz = type_size(src->types[i]);
            ST_ARGH(sz > 0 && dst->types[i] == src->types[i], "filter_nan: bad or mismatched column type");
            dcols[i] = ws(c, "h.fn" + std::to_string(i), n * sz + 16);
            b.add(static_cast<const char *>(src->cols[i]), static_cast<char *>(dcols[i]), n * sz);
        }
        b.h2d();
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
            b.add_d2h(static_cast<char *>(dst->cols[i]), static_cast<const char *>(ocols[i]),
                      m * type_size(src->types[i]));
        b.d2h();
        *out_m = m;
    });
}

int st_morton_order(st_ctx *c, const float *x, const float *y, const float *z, uint32_t *idx, uint64_t n) {
    return guarded_h([&] {
        ST_ARGH(c && ((x && y && z && idx) || n == 0), "NULL argument");
        if (n == 0) return;
        use_device(c);
        Batch b{c};
        float *dx = to_dev(b, "h.mx", x, n), *dy = to_dev(b, "h.my", y, n), *dz = to_dev(b, "h.mz", z, n);
        uint32_t *di = to_dev(b, "h.mi", idx, n);
        b.h2d();
        morton_order_dev(c, dx, dy, dz, di, n);
        b.add_d2h(idx, di, n);
        b.d2h();
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
        Batch b{c};
        uint32_t *dord = to_dev(b, "h.cord", order, n);
        b.h2d();
        auto *dchunk = wsT<float>(c, "h.cchunk", nch * 18);
        auto *dvert = wsT<uint32_t>(c, "h.cvert", n * 4);
        auto *dsh = wsT<uint8_t>(c, "h.csh", n * (uint64_t)nsh + 1);
        pack_compressed_dev(c, &d.t, dord, dchunk, dvert, dsh);
        b.add_d2h(chunk, dchunk, nch * 18);
        b.add_d2h(vertex, dvert, n * 4);
        if (nsh) b.add_d2h(sh, dsh, n * (uint64_t)nsh);
        b.d2h();
    });
}

int st_kmeans(st_ctx *c, const float *const *cols, int32_t d, uint64_t n, int32_t k, int32_t iters,
              const double *draws, uint64_t ndraws, uint64_t *used, float *centroids, uint32_t *labels) {
    return guarded_h([&] {
        ST_ARGH(c && cols && d > 0 && k > 0 && centroids && labels, "bad argument");
        use_device(c);
        std::vector<const float *> dc(d);
        Batch b{c};
        for (int j = 0; j < d; ++j) dc[j] = to_dev(b, "h.k" + std::to_string(j), cols[j], n);
        b.h2d();
        const uint64_t kk = n < (uint64_t)k ? n : (uint64_t)k;
        auto *dcen = wsT<float>(c, "h.kcen", (size_t)d * (k > (int)kk ? k : kk));
        auto *dlab = wsT<uint32_t>(c, "h.klab", n);
        const uint64_t u = kmeans_dev(c, dc.data(), d, n, k, iters, draws, ndraws, dcen, dlab);
        b.add_d2h(centroids, dcen, (size_t)d * kk);
        b.add_d2h(labels, dlab, n);
        b.d2h();
        if (used) *used = u;
    });
}

int st_cluster1d(st_ctx *c, const float *const *cols, int32_t ncols, uint64_t n, int32_t iters, const double *draws,
                 uint64_t ndraws, uint64_t *used, float *centroids256, uint8_t *labels) {
    return guarded_h([&] {
        ST_ARGH(c && cols && ncols > 0 && centroids256 && labels, "bad argument");
        use_device(c);
        std::vector<const float *> dc(ncols);
        Batch b{c};
        for (int j = 0; j < ncols; ++j) dc[j] = to_dev(b, "h.1d" + std::to_string(j), cols[j], n);
        b.h2d();
        auto *dcen = wsT<float>(c, "h.1dcen", 256);
        auto *dlab = wsT<uint8_t>(c, "h.1dlab", n * (uint64_t)ncols);
        const uint64_t u = cluster1d_dev(c, dc.data(), ncols, n, iters, draws, ndraws, dcen, dlab);
        b.add_d2h(centroids256, dcen, 256);
        b.add_d2h(labels, dlab, n * (uint64_t)ncols);
        b.d2h();
        if (used) *used = u;
    });
}

int st_sog(st_ctx *c, const st_table *t, int32_t iters, const double *draws, uint64_t ndraws, uint64_t *used,
           st_sog_meta *meta, const st_sog_textures *out) {
    if (int rc = apply_env_devices()) return rc;
    if (auto g = default_group()) return st_group_sog(g.get(), &t, 1, nullptr, iters, draws, ndraws, used, meta, out);
    return guarded_h([&] {
        ST_ARGH(c && t && meta && out, "NULL argument");
        use_device(c);
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
        uint64_t u = 0;
        run_host_sog(c, t, sog_columns(), "h.s", [&](const st_table *dtab) {
            u = sog_dev(c, dtab, iters, draws, ndraws, meta, &dt);
            spec_gate(c);
        });
        Batch b{c};
        b.add_d2h(out->means_l, dt.means_l, tex);
        b.add_d2h(out->means_u, dt.means_u, tex);
        b.add_d2h(out->quats, dt.quats, tex);
        b.add_d2h(out->scales, dt.scales, tex);
        b.add_d2h(out->sh0, dt.sh0, tex);
        if (C) {
            ST_ARGH(out->shn_labels && out->shn_centroids, "sog: shN outputs are NULL");
            b.add_d2h(out->shn_labels, dt.shn_labels, tex);
            b.add_d2h(out->shn_centroids, dt.shn_centroids, (uint64_t)cw * chh * 4);
        }
        b.d2h();
        if (used) *used = u;
    });
}

// writeSog to a .sog bundle (write-sog.ts:110-370 with the ZipWriter of :112-114):
// the archive bytes, malloc'd (st_free)
int st_sog_bundle(st_ctx *c, const st_table *t, int32_t iters, const double *draws, uint64_t ndraws, uint64_t *used,
                  uint16_t dos_time, uint16_t dos_date, uint8_t **out, uint64_t *out_size) {
    if (int rc = apply_env_devices()) return rc;
    if (auto g = default_group())
        return st_group_sog_bundle(g.get(), &t, 1, nullptr, iters, draws, ndraws, used, dos_time, dos_date, out, out_size);
    return guarded_h([&] {
        ST_ARGH(c && t && out && out_size, "NULL argument");
        use_device(c);
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
        uint64_t u = 0;
        run_host_sog(c, t, sog_columns(), "h.s", [&](const st_table *dtab) {
            u = sog_dev(c, dtab, iters, draws, ndraws, &meta, &dt);
            spec_gate(c);
        });
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

int st_sog_file(st_ctx *c, const st_table *t, int32_t iters, const double *draws, uint64_t ndraws, uint64_t *used,
                int32_t fd, uint16_t dos_time, uint16_t dos_date, uint64_t *size) {
    if (int rc = apply_env_devices()) return rc;
    if (auto g = default_group()) {  // rows sharded over GPUs: the group's archive, then one write
        if (int rc = guarded_h([&] {
                ST_ARGH(size, "bad argument");
                sog_file_check(fd);
            }))
            return rc;
        uint8_t *zip = nullptr;
        uint64_t nb = 0;
        if (int rc = st_group_sog_bundle(g.get(), &t, 1, nullptr, iters, draws, ndraws, used, dos_time, dos_date, &zip,
                                         &nb))
            return rc;
        const int rc = guarded_h([&] {  // the same writer as the one-GPU path: from offset 0, then truncated
            write_at(fd, zip, nb, 0);
            sog_file_truncate(fd, nb);
            *size = nb;
        });
        std::free(zip);
        return rc;
    }
    return guarded_h([&] {
        ST_ARGH(c && t && size && fd >= 0, "bad argument");
        use_device(c);
        sog_file_check(fd);
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
        uint64_t u = 0;
        run_host_sog(c, t, sog_columns(), "h.s", [&](const st_table *dtab) {
            u = sog_file_dev(c, dtab, iters, draws, ndraws, &meta, &dt, fd, dos_time, dos_date, size);
        });
        if (used) *used = u;
    });
}

}  // extern "C"
