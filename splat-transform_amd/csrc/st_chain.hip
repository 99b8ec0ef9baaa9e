// st_chain.hip -- processDataTable (process.ts:64-145) over a table resident in HBM, and the
// CLI's `in.ply [actions] out.compressed.ply` (index.ts:463-496 -> writeCompressedPly,
// write-compressed-ply.ts:31-115) as one call: the table crosses PCIe once in each direction
// (columns up, packed chunk / vertex / sh bytes down) instead of once per action.
//
// The chain holds the current table as (name, type, device pointer) columns.  A transform
// updates float32 columns in place; a filter gathers the survivors into the other of two
// workspace generations (ping-pong), so a long action list needs at most two copies of the
// table beside the input.
#include <unistd.h>

#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <exception>
#include <mutex>
#include <thread>

#include <chrono>

#include "st_internal.h"
#include "st_typed.h"
#include "st_webp.h"

namespace st {
namespace {

struct ChainCol {
    std::string name;
    int32_t type;
    void *ptr;
};

struct Chain {
    st_ctx *c;
    uint64_t n = 0;
    std::vector<ChainCol> cols;
    int gen = 0;                  // workspace generation the next filter writes
    std::string tag = "chain";    // workspace slot prefix (several chains alive at once)

    // views over the current columns (rebuilt on demand; pointers stay valid until the next change)
    std::vector<const char *> names;
    std::vector<int32_t> types;
    std::vector<void *> ptrs;
    std::vector<float *> fptrs;
    std::vector<const char *> fnames;
    st_ttable tt{};
    st_table ft{};

    const st_ttable *typed() {
        names.clear(), types.clear(), ptrs.clear();
        for (auto &k : cols) names.push_back(k.name.c_str()), types.push_back(k.type), ptrs.push_back(k.ptr);
        tt = st_ttable{n, (int32_t)cols.size(), names.data(), types.data(), ptrs.data()};
        return &tt;
    }
    // the float32 columns as an st_table (the transform / pack kernels read columns by name)
    const st_table *f32() {
        fnames.clear(), fptrs.clear();
        for (auto &k : cols)
            if (k.type == ST_PLY_FLOAT) fnames.push_back(k.name.c_str()), fptrs.push_back(static_cast<float *>(k.ptr));
        ft = st_table{n, (int32_t)fptrs.size(), fnames.data(), fptrs.data()};
        return &ft;
    }
    bool has(const std::string &nm) const {
        for (auto &k : cols)
            if (k.name == nm) return true;
        return false;
    }
    // the kernels read these by name from the float32 columns: a same-named column of another
    // type would be silently skipped (the reference reads any type through getRow)
    void require_f32(const std::string &nm, const char *what) const {
        for (auto &k : cols)
            if (k.name == nm && k.type != ST_PLY_FLOAT)
                throw Error(ST_ERR_UNSUPPORTED, std::string(what) + ": column " + nm + " is not float32");
    }

    void gather(const uint32_t *idx, uint64_t m) {
        const st_ttable *src = typed();
        std::vector<void *> dst(cols.size());
        for (size_t i = 0; i < cols.size(); ++i)
            dst[i] = ws(c, tag + ".g" + std::to_string(gen) + "." + std::to_string(i), m * type_size(cols[i].type) + 16);
        st_ttable d = *src;
        d.n = m;
        d.cols = dst.data();
        permute_rows_tdev(c, src, idx, m, &d);
        for (size_t i = 0; i < cols.size(); ++i) cols[i].ptr = dst[i];
        n = m;
        gen ^= 1;
    }
};

int band_coeffs(const std::vector<ChainCol> &cols) {
    // { '9': 1, '24': 2, '-1': 3 }[shNames.findIndex(v => !dataTable.hasColumn(v))] ?? 0
    int first_missing = -1;
    for (int i = 0; i < 45 && first_missing < 0; ++i) {
        const std::string nm = "f_rest_" + std::to_string(i);
        bool hit = false;
        for (auto &k : cols) hit = hit || k.name == nm;
        if (!hit) first_missing = i;
    }
    return first_missing == 9 ? 3 : first_missing == 24 ? 8 : first_missing == -1 ? 15 : 0;
}

void run_actions(Chain &ch, const st_action *actions, int nactions) {
    const int in_coeffs = band_coeffs(ch.cols);  // filterBands reads the ORIGINAL table (process.ts:111)
    for (int a = 0; a < nactions; ++a) {
        const st_action &act = actions[a];
        switch (act.kind) {
            case ST_ACTION_TRANSFORM:
                // every column type, as getRow / setRow (transform.ts:24-63)
                transform_tdev(ch.c, ch.typed(), &act.transform);
                break;
            case ST_ACTION_FILTER_NAN:
            case ST_ACTION_FILTER_VALUE: {
                if (ch.n == 0) break;
                auto *idx = wsT<uint32_t>(ch.c, ch.tag + ".idx", ch.n);
                const uint64_t m = act.kind == ST_ACTION_FILTER_NAN
                                       ? filter_finite_tdev(ch.c, ch.typed(), idx)
                                       : filter_value_tdev(ch.c, ch.typed(), act.column, act.compare, act.value, idx);
                if (m != ch.n) ch.gather(idx, m);  // all rows kept: permuteRows by the identity
                break;
            }
            case ST_ACTION_FILTER_BANDS: {
                ST_REQUIRE(act.bands >= 0 && act.bands <= 3, ST_ERR_ARG, "filterBands: bands must be 0..3");
                static const int coeffs[4] = {0, 3, 8, 15};
                const int out_coeffs = coeffs[act.bands];
                if (out_coeffs >= in_coeffs) break;  // outputBands < inputBands only (:115)
                std::vector<ChainCol> next;
                for (auto &k : ch.cols) {
                    int hit = -1, to = -1;
                    for (int i = 0; i < in_coeffs && hit < 0; ++i)
                        for (int j = 0; j < 3 && hit < 0; ++j)
                            if (k.name == "f_rest_" + std::to_string(i + j * in_coeffs)) {
                                hit = 1;
                                if (i < out_coeffs) to = i + j * out_coeffs;
                            }
                    if (hit < 0) next.push_back(k);
                    else if (to >= 0) next.push_back(ChainCol{"f_rest_" + std::to_string(to), k.type, k.ptr});
                }
                ch.cols.swap(next);
                break;
            }
            case ST_ACTION_PARAM:
                break;
            default:
                throw Error(ST_ERR_ARG, "process: unknown action kind " + std::to_string(act.kind));
        }
    }
}

// writeCompressedPly's device part on the processed table: Morton order of the identity
// (write-compressed-ply.ts:59-64), then the chunk loop
// (any column types: the chunk members go through CompressedChunk's Float32Arrays
// (compressed-chunk.ts:28-41), the ordering and the SH bytes read the row's JS numbers
// (ordering.ts:32-47, write-compressed-ply.ts:85))
const char *const SH_NAMES[45] = {
    "f_rest_0",  "f_rest_1",  "f_rest_2",  "f_rest_3",  "f_rest_4",  "f_rest_5",  "f_rest_6",  "f_rest_7",  "f_rest_8",
    "f_rest_9",  "f_rest_10", "f_rest_11", "f_rest_12", "f_rest_13", "f_rest_14", "f_rest_15", "f_rest_16", "f_rest_17",
    "f_rest_18", "f_rest_19", "f_rest_20", "f_rest_21", "f_rest_22", "f_rest_23", "f_rest_24", "f_rest_25", "f_rest_26",
    "f_rest_27", "f_rest_28", "f_rest_29", "f_rest_30", "f_rest_31", "f_rest_32", "f_rest_33", "f_rest_34", "f_rest_35",
    "f_rest_36", "f_rest_37", "f_rest_38", "f_rest_39", "f_rest_40", "f_rest_41", "f_rest_42", "f_rest_43", "f_rest_44"};

void compressed_tail(Chain &ch, float *chunk, uint32_t *vertex, uint8_t *sh, int32_t *out_coeffs) {
    static const char *pcols[] = {"x", "y", "z", "scale_0", "scale_1", "scale_2", "f_dc_0",
                                  "f_dc_1", "f_dc_2", "opacity", "rot_0", "rot_1", "rot_2", "rot_3"};
    const int C = band_coeffs(ch.cols);
    *out_coeffs = C;
    if (ch.n == 0) return;
    const st_ttable *tt = ch.typed();
    std::vector<const char *> fn;
    std::vector<float *> fp;
    TCol xyz[3];
    for (int i = 0; i < 14; ++i) {
        const TCol col = tcol_or_null(tt, pcols[i]);
        ST_REQUIRE(col.p, ST_ERR_ARG, std::string("pack_compressed: missing column ") + pcols[i]);
        if (i < 3) xyz[i] = col;
        fn.push_back(pcols[i]);
        fp.push_back(const_cast<float *>(as_f32_dev(ch.c, col, ch.n, ch.tag + ".m32." + std::to_string(i))));
    }
    bool sh32 = true;
    std::vector<const double *> sh64;
    for (int i = 0; i < 3 * C; ++i) sh32 = sh32 && tcol_or_null(tt, SH_NAMES[i]).t == ST_PLY_FLOAT;
    for (int i = 0; i < 3 * C; ++i) {
        const TCol col = tcol_or_null(tt, SH_NAMES[i]);
        if (sh32) fn.push_back(SH_NAMES[i]), fp.push_back(static_cast<float *>(col.p));
        else sh64.push_back(as_f64_dev(ch.c, col, ch.n, ch.tag + ".sh64." + std::to_string(i)));
    }
    const st_table t{ch.n, (int32_t)fp.size(), fn.data(), fp.data()};
    auto *order = wsT<uint32_t>(ch.c, "chain.order", ch.n);
    iota_u32(ch.c, order, ch.n);
    const void *xp[3] = {xyz[0].p, xyz[1].p, xyz[2].p};
    const int32_t xt[3] = {xyz[0].t, xyz[1].t, xyz[2].t};
    morton_order_tdev(ch.c, xp, xt, order, ch.n);
    pack_compressed_dev(ch.c, &t, order, chunk, vertex, sh, sh32 ? nullptr : sh64.data(), C);
}

void check_src(const st_ttable *src) {
    ST_REQUIRE(src->ncol >= 0 && (src->ncol == 0 || (src->names && src->types && src->cols)), ST_ERR_ARG,
               "process: bad table");
    for (int i = 0; i < src->ncol; ++i) {
        ST_REQUIRE(type_size(src->types[i]) > 0, ST_ERR_ARG, "process: bad column type");
        ST_REQUIRE(src->n == 0 || src->cols[i], ST_ERR_ARG, "process: NULL column");
    }
}

// upload the host table once
void upload_chain(st_ctx *c, const st_ttable *src, Chain &ch) {
    ch.n = src->n;
    std::vector<HostXfer> up;
    for (int i = 0; i < src->ncol; ++i) {
        const int sz = type_size(src->types[i]);
        void *d = ws(c, "chain.in." + std::to_string(i), src->n * sz + 16);
        up.push_back(HostXfer{src->cols[i], d, src->n * sz});
        ch.cols.push_back(ChainCol{src->names[i], src->types[i], d});
    }
    staged_h2d(c, up);
}

// the element's rows straight from the file into HBM columns (page cache -> pinned -> HBM,
// st_dev_ply_read); element < 0 selects the one named "vertex" (read-ply.ts's splat element)
void ply_chain(st_ctx *c, int fd, const st_ply_header *h, int element, Chain &ch) {
    if (element < 0)
        for (int e = 0; e < h->nelements && element < 0; ++e)
            if (std::strcmp(h->elements[e].name, "vertex") == 0) element = e;
    ST_REQUIRE(element >= 0 && element < h->nelements, ST_ERR_ARG, "ply: no such element");
    const st_ply_element &el = h->elements[element];
    std::vector<void *> cols(el.nprops);
    for (int p = 0; p < el.nprops; ++p) {
        cols[p] = ws(c, "chain.in." + std::to_string(p), el.count * type_size(el.props[p].type) + 16);
        ch.cols.push_back(ChainCol{el.props[p].name, el.props[p].type, cols[p]});
    }
    ch.n = el.count;
    ply_read_dev(c, fd, *h, element, cols.data());
}

// the processed table as the multi-GPU writeSog takes it: float32 columns by name (the sharded
// path moves float32 columns only; a single device takes every type through sog_tdev)
const st_table *sog_view(Chain &ch) {
    static const char *scols[] = {"x", "y", "z", "scale_0", "scale_1", "scale_2", "f_dc_0", "f_dc_1", "f_dc_2",
                                  "opacity", "rot_0", "rot_1", "rot_2", "rot_3"};
    for (auto *nm : scols) ch.require_f32(nm, "multi-GPU writeSog");
    for (int i = 0; i < 45; ++i) ch.require_f32("f_rest_" + std::to_string(i), "multi-GPU writeSog");
    return ch.f32();
}

// device textures of writeSog for n rows of band C (workspace slots h.s.*)
st_sog_textures sog_textures(st_ctx *c, uint64_t n, int C, uint64_t *tex_bytes, uint64_t *cen_bytes) {
    int32_t W, H, pal, cw, chh;
    ST_REQUIRE(st_sog_geometry(n, C, &W, &H, &pal, &cw, &chh) == ST_OK, ST_ERR_ARG, "sog: empty table");
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
    *tex_bytes = tex;
    *cen_bytes = (uint64_t)cw * chh * 4;
    return dt;
}



// ---- writeCompressedPly into a file (write-compressed-ply.ts:31-115 + the CLI's write) --------
// the header text of write-compressed-ply.ts:35-54
std::string compressed_ply_header(uint64_t m, int C, const char *version) {
    static const char *chunk_props[18] = {"min_x", "min_y", "min_z", "max_x", "max_y", "max_z",
                                          "min_scale_x", "min_scale_y", "min_scale_z", "max_scale_x", "max_scale_y",
                                          "max_scale_z", "min_r", "min_g", "min_b", "max_r", "max_g", "max_b"};
    static const char *vertex_props[4] = {"packed_position", "packed_rotation", "packed_scale", "packed_color"};
    std::string h = "ply\nformat binary_little_endian 1.0\ncomment Generated by splat-transform ";
    h += (version && *version) ? version : "0.10.1";
    h += "\nelement chunk " + std::to_string((m + 255) / 256) + "\n";
    for (auto *p : chunk_props) h += std::string("property float ") + p + "\n";
    h += "element vertex " + std::to_string(m) + "\n";
    for (auto *p : vertex_props) h += std::string("property uint ") + p + "\n";
    if (C) {
        h += "element sh " + std::to_string(m) + "\n";
        for (int i = 0; i < 3 * C; ++i) h += "property uchar f_rest_" + std::to_string(i) + "\n";
    }
    return h + "end_header\n";
}

// the device arrays to fd at offsets from its position: pinned slots filled by device-to-host copies on
// the context's stream while a host thread writes the slot before (ext4 / xfs serialise buffered
// writes to one file, so one writer); the file ends at the last byte
uint64_t compressed_ply_to_file(st_ctx *c, uint64_t m, int C, const float *dchunk, const uint32_t *dvert,
                                const uint8_t *dsh, int fd, const char *version) {
    const std::string head = compressed_ply_header(m, C, version);
    // from the descriptor's position, as the reference's FileHandle.write calls go (the CLI's
    // fresh output: 0), which is left at the end of what was written
    const off_t pos = lseek(fd, 0, SEEK_CUR);
    ST_REQUIRE(pos >= 0, ST_ERR_ARG, "compressed ply file: the descriptor has no position");
    const uint64_t base = (uint64_t)pos;
    write_at(fd, reinterpret_cast<const uint8_t *>(head.data()), head.size(), base);
    const uint64_t nch = (m + 255) / 256;
    struct Region {
        const uint8_t *dev;
        uint64_t bytes, off;
    };
    std::vector<Region> rs;
    uint64_t off = base + head.size();
    for (const Region &r : {Region{reinterpret_cast<const uint8_t *>(dchunk), nch * 72, 0},
                            Region{reinterpret_cast<const uint8_t *>(dvert), m * 16, 0},
                            Region{dsh, C ? m * 3 * (uint64_t)C : 0, 0}}) {
        if (r.bytes) rs.push_back({r.dev, r.bytes, off});
        off += r.bytes;
    }
    const uint64_t total = off;
    constexpr int SLOTS = 4;
    uint64_t slot = 32ull << 20;
    if (const char *e = std::getenv("ST_CPF_SLOT_MB")) slot = std::max<uint64_t>(1, std::strtoull(e, nullptr, 10)) << 20;
    auto *ring = static_cast<uint8_t *>(pinned_slot(c, "cpf.ring", SLOTS * slot));
    struct Piece {
        int s;
        uint64_t bytes, off;
        hipEvent_t ev;
    };
    std::mutex mu;
    std::condition_variable cv;
    std::deque<Piece> q;
    bool busy[SLOTS] = {}, fin = false;
    std::exception_ptr err;
    std::thread writer([&] {
        for (;;) {
            Piece p;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return fin || !q.empty(); });
                if (q.empty()) return;
                p = q.front();
                q.pop_front();
            }
            try {
                const hipError_t e = hipEventSynchronize(p.ev);
                (void)hipEventDestroy(p.ev);
                ST_HIP(e);
                bool skip;
                {
                    std::lock_guard<std::mutex> lk(mu);
                    skip = (bool)err;
                }
                if (!skip) write_at(fd, ring + p.s * slot, p.bytes, p.off);
            } catch (...) {
                std::lock_guard<std::mutex> lk(mu);
                if (!err) err = std::current_exception();
            }
            {
                std::lock_guard<std::mutex> lk(mu);
                busy[p.s] = false;
            }
            cv.notify_all();
        }
    });
    auto stop = [&] {
        {
            std::lock_guard<std::mutex> lk(mu);
            fin = true;
        }
        cv.notify_all();
        if (writer.joinable()) writer.join();
    };
    try {
        int k = 0;
        for (const Region &r : rs)
            for (uint64_t o = 0; o < r.bytes; o += slot, ++k) {
                const int sidx = k % SLOTS;
                const uint64_t nb = std::min(slot, r.bytes - o);
                {
                    std::unique_lock<std::mutex> lk(mu);
                    cv.wait(lk, [&] { return !busy[sidx] || err; });
                    if (err) break;
                    busy[sidx] = true;
                }
                hipEvent_t ev;
                ST_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
                ST_HIP(hipMemcpyAsync(ring + sidx * slot, r.dev + o, nb, hipMemcpyDeviceToHost, c->stream));
                ST_HIP(hipEventRecord(ev, c->stream));
                {
                    std::lock_guard<std::mutex> lk(mu);
                    q.push_back({sidx, nb, r.off + o, ev});
                }
                cv.notify_all();
            }
    } catch (...) {
        {
            std::lock_guard<std::mutex> lk(mu);
            if (!err) err = std::current_exception();
        }
    }
    stop();
    if (err) std::rethrow_exception(err);
    sog_file_truncate(fd, total);
    ST_REQUIRE(lseek(fd, (off_t)total, SEEK_SET) == (off_t)total, ST_ERR_ARG, "compressed ply file: lseek failed");
    return total - base;
}

#define ST_REQUIRE_RC(cond, msg)           \
    do {                                   \
        if (!(cond)) {                     \
            set_last_error(msg);           \
            return ST_ERR_ARG;             \
        }                                  \
    } while (0)

// processDataTable + writeSog on a table the loader puts in the chain: the .sog archive
// (out / out_size) or the textures and meta on the host (tex_meta / tex_out).  One device takes
// every column type (sog_tdev); with the st_set_devices group the processed float32 columns are
// sharded over it from the host.
template <typename Load>
int sog_chain(st_ctx *c, Load load, const st_action *actions, int32_t nactions, int32_t iters, const double *draws,
              uint64_t ndraws, uint64_t *used, uint16_t dos_time, uint16_t dos_date, uint8_t **out,
              uint64_t *out_size, st_sog_meta *tex_meta, const st_sog_textures *tex_out) {
    if (int rc = apply_env_devices()) return rc;
    const auto group = default_group();  // held for the whole call
    std::vector<std::vector<float>> host;  // multi-GPU: the processed columns, sharded from the host
    std::vector<float *> hcols;
    std::vector<std::string> hnames;
    std::vector<const char *> hcn;
    st_table ht{};
    int rc = guard([&] {
        ST_REQUIRE(c && ((out && out_size) || (tex_meta && tex_out)), ST_ERR_ARG, "NULL argument");
        ST_REQUIRE(actions || nactions == 0, ST_ERR_ARG, "NULL argument");
        use_device(c);
        Chain ch{c};
        load(ch);
        run_actions(ch, actions, nactions);
        if (group) {
            const st_table *t = sog_view(ch);
            std::vector<HostXfer> down;
            for (int i = 0; i < t->ncol; ++i) {
                host.emplace_back(t->n);
                hnames.push_back(t->names[i]);
                down.push_back(HostXfer{host.back().data(), t->cols[i], t->n * 4});
            }
            staged_d2h(c, down);
            for (size_t i = 0; i < host.size(); ++i) hcols.push_back(host[i].data()), hcn.push_back(hnames[i].c_str());
            ht = st_table{t->n, t->ncol, hcn.data(), hcols.data()};
            return;
        }
        const int C = band_coeffs(ch.cols);
        uint64_t tex, cbytes;
        const st_sog_textures dt = sog_textures(c, ch.n, C, &tex, &cbytes);
        st_sog_meta meta{};
        const uint64_t u = sog_tdev(c, ch.typed(), iters, draws, ndraws, &meta, &dt);
        if (tex_out) {
            std::vector<HostXfer> down;
            for (auto pr : {std::make_pair(tex_out->means_l, dt.means_l), std::make_pair(tex_out->means_u, dt.means_u),
                            std::make_pair(tex_out->quats, dt.quats), std::make_pair(tex_out->scales, dt.scales),
                            std::make_pair(tex_out->sh0, dt.sh0)}) {
                ST_REQUIRE(pr.first, ST_ERR_ARG, "sog: texture output is NULL");
                down.push_back(HostXfer{pr.first, pr.second, tex});
            }
            if (C) {
                ST_REQUIRE(tex_out->shn_labels && tex_out->shn_centroids, ST_ERR_ARG, "sog: shN outputs are NULL");
                down.push_back(HostXfer{tex_out->shn_labels, dt.shn_labels, tex});
                down.push_back(HostXfer{tex_out->shn_centroids, dt.shn_centroids, cbytes});
            }
            staged_d2h(c, down);
            *tex_meta = meta;
        } else {
            const uint8_t *view;
            uint64_t nb;
            sog_bundle_dev(c, meta, ch.n, dt, dos_time, dos_date, &view, &nb);
            uint8_t *buf = (uint8_t *)std::malloc(nb);
            ST_REQUIRE(buf, ST_ERR_NOMEM, "sog bundle: host allocation failed");
            std::memcpy(buf, view, nb);
            *out = buf;
            *out_size = nb;
        }
        if (used) *used = u;
    });
    if (rc != ST_OK || !ht.ncol) return rc;
    const st_table *tp = &ht;
    if (tex_out) return st_group_sog(group.get(), &tp, 1, nullptr, iters, draws, ndraws, used, tex_meta, tex_out);
    return st_group_sog_bundle(group.get(), &tp, 1, nullptr, iters, draws, ndraws, used, dos_time, dos_date, out,
                               out_size);
}

}  // namespace

// processDataTable on a device float32 table (transforms in place, filters into workspace slots
// under `tag`): the processed table's columns in `out`
void chain_apply_f32(st_ctx *c, const st_table *in, const st_action *actions, int nactions, const std::string &tag,
                     ProcessedF32 &out) {
    Chain ch{c};
    ch.tag = tag;
    ch.n = in->n;
    for (int i = 0; i < in->ncol; ++i) ch.cols.push_back(ChainCol{in->names[i], ST_PLY_FLOAT, in->cols[i]});
    run_actions(ch, actions, nactions);
    out.names.clear();
    out.cn.clear();
    out.cols.clear();
    for (auto &k : ch.cols) out.names.push_back(k.name), out.cols.push_back(static_cast<float *>(k.ptr));
    for (auto &nm : out.names) out.cn.push_back(nm.c_str());
    out.t = st_table{ch.n, (int32_t)out.cols.size(), out.cn.data(), out.cols.data()};
}

}  // namespace st

using namespace st;

extern "C" {

int st_process(st_ctx *c, const st_ttable *src, const st_action *actions, int32_t nactions, const st_ttable *dst,
               uint64_t *out_m) {
    return guard([&] {
        ST_REQUIRE(c && src && dst && out_m && (actions || nactions == 0), ST_ERR_ARG, "NULL argument");
        check_src(src);
        use_device(c);
        Chain ch{c};
        upload_chain(c, src, ch);
        run_actions(ch, actions, nactions);
        std::vector<int> from(dst->ncol, -1);
        for (int j = 0; j < dst->ncol; ++j) {
            for (size_t i = 0; i < ch.cols.size() && from[j] < 0; ++i)
                if (ch.cols[i].name == dst->names[j] && ch.cols[i].type == dst->types[j]) from[j] = (int)i;
            ST_REQUIRE(from[j] >= 0, ST_ERR_ARG, std::string("process: result has no column ") + dst->names[j]);
        }
        std::vector<HostXfer> down;
        for (int j = 0; j < dst->ncol; ++j)
            down.push_back(HostXfer{dst->cols[j], ch.cols[from[j]].ptr, ch.n * type_size(dst->types[j])});
        staged_d2h(c, down);
        *out_m = ch.n;
    });
}

int st_compressed_ply(st_ctx *c, const st_ttable *src, const st_action *actions, int32_t nactions, float *chunk,
                      uint32_t *vertex, uint8_t *sh, uint64_t *out_m, int32_t *out_sh_coeffs) {
    return guard([&] {
        ST_REQUIRE(c && src && out_m && out_sh_coeffs && (actions || nactions == 0), ST_ERR_ARG, "NULL argument");
        check_src(src);
        use_device(c);
        Chain ch{c};
        upload_chain(c, src, ch);
        run_actions(ch, actions, nactions);
        const uint64_t m = ch.n, nch = (m + 255) / 256;
        ST_REQUIRE(m == 0 || (chunk && vertex), ST_ERR_ARG, "compressed_ply: NULL output");
        auto *dchunk = wsT<float>(c, "chain.chunk", nch * 18);
        auto *dvert = wsT<uint32_t>(c, "chain.vert", m * 4);
        const int Cmax = band_coeffs(ch.cols);
        auto *dsh = wsT<uint8_t>(c, "chain.sh", m * 3 * (uint64_t)Cmax + 1);
        int32_t C = 0;
        compressed_tail(ch, dchunk, dvert, dsh, &C);
        ST_REQUIRE(C == 0 || m == 0 || sh, ST_ERR_ARG, "compressed_ply: sh output is NULL");
        std::vector<HostXfer> down;
        if (m) {
            down.push_back(HostXfer{chunk, dchunk, nch * 18 * 4});
            down.push_back(HostXfer{vertex, dvert, m * 16});
            if (C) down.push_back(HostXfer{sh, dsh, m * 3 * (uint64_t)C});
        }
        staged_d2h(c, down);
        *out_m = m;
        *out_sh_coeffs = C;
    });
}

int st_dev_compressed_ply(st_ctx *c, const st_ttable *src, const st_action *actions, int32_t nactions,
                          float *chunk, uint32_t *vertex, uint8_t *sh, uint64_t *out_m, int32_t *out_sh_coeffs) {
    return guard([&] {
        ST_REQUIRE(c && src && out_m && out_sh_coeffs && (actions || nactions == 0), ST_ERR_ARG, "NULL argument");
        check_src(src);
        use_device(c);
        Chain ch{c};
        ch.n = src->n;
        for (int i = 0; i < src->ncol; ++i) ch.cols.push_back(ChainCol{src->names[i], src->types[i], src->cols[i]});
        run_actions(ch, actions, nactions);
        ST_REQUIRE(ch.n == 0 || (chunk && vertex), ST_ERR_ARG, "compressed_ply: NULL output");
        int32_t C = 0;
        if (band_coeffs(ch.cols) && ch.n) ST_REQUIRE(sh, ST_ERR_ARG, "compressed_ply: sh output is NULL");
        compressed_tail(ch, chunk, vertex, sh, &C);
        *out_m = ch.n;
        *out_sh_coeffs = C;
    });
}

int st_ply_compressed_ply(st_ctx *c, int32_t fd, const st_ply_header *h, int32_t element, const st_action *actions,
                          int32_t nactions, float *chunk, uint32_t *vertex, uint8_t *sh, uint64_t *out_m,
                          int32_t *out_sh_coeffs) {
    return guard([&] {
        ST_REQUIRE(c && h && fd >= 0 && out_m && out_sh_coeffs && (actions || nactions == 0), ST_ERR_ARG,
                   "NULL argument");
        use_device(c);
        Chain ch{c};
        ply_chain(c, fd, h, element, ch);
        run_actions(ch, actions, nactions);
        const uint64_t m = ch.n, nch = (m + 255) / 256;
        ST_REQUIRE(m == 0 || (chunk && vertex), ST_ERR_ARG, "compressed_ply: NULL output");
        auto *dchunk = wsT<float>(c, "chain.chunk", nch * 18);
        auto *dvert = wsT<uint32_t>(c, "chain.vert", m * 4);
        auto *dsh = wsT<uint8_t>(c, "chain.sh", m * 3 * (uint64_t)band_coeffs(ch.cols) + 1);
        int32_t C = 0;
        compressed_tail(ch, dchunk, dvert, dsh, &C);
        ST_REQUIRE(C == 0 || m == 0 || sh, ST_ERR_ARG, "compressed_ply: sh output is NULL");
        std::vector<HostXfer> down;
        if (m) {
            down.push_back(HostXfer{chunk, dchunk, nch * 18 * 4});
            down.push_back(HostXfer{vertex, dvert, m * 16});
            if (C) down.push_back(HostXfer{sh, dsh, m * 3 * (uint64_t)C});
        }
        staged_d2h(c, down);
        *out_m = m;
        *out_sh_coeffs = C;
    });
}

int st_ply_compressed_ply_file(st_ctx *c, int32_t fd, const st_ply_header *h, int32_t element,
                               const st_action *actions, int32_t nactions, int32_t out_fd, const char *version,
                               uint64_t *out_m, int32_t *out_sh_coeffs, uint64_t *size) {
    return guard([&] {
        ST_REQUIRE(c && h && fd >= 0 && out_m && out_sh_coeffs && size && (actions || nactions == 0), ST_ERR_ARG,
                   "NULL argument");
        sog_file_check(out_fd);
        use_device(c);
        using clk = std::chrono::steady_clock;
        const auto t0 = clk::now();
        Chain ch{c};
        ply_chain(c, fd, h, element, ch);
        ST_HIP(hipStreamSynchronize(c->stream));  // (ST_DEBUG's stamps: the ingest alone)
        const auto t1 = clk::now();
        run_actions(ch, actions, nactions);
        const uint64_t m = ch.n, nch = (m + 255) / 256;
        auto *dchunk = wsT<float>(c, "chain.chunk", nch * 18);
        auto *dvert = wsT<uint32_t>(c, "chain.vert", m * 4);
        auto *dsh = wsT<uint8_t>(c, "chain.sh", m * 3 * (uint64_t)band_coeffs(ch.cols) + 1);
        int32_t C = 0;
        compressed_tail(ch, dchunk, dvert, dsh, &C);
        ST_HIP(hipStreamSynchronize(c->stream));
        const auto t2 = clk::now();
        *size = compressed_ply_to_file(c, m, C, dchunk, dvert, dsh, out_fd, version);
        *out_m = m;
        *out_sh_coeffs = C;
        if (std::getenv("ST_DEBUG")) {
            const auto ms = [](clk::time_point a, clk::time_point b) {
                return std::chrono::duration<double, std::milli>(b - a).count();
            };
            fprintf(stderr, "[st cply file] ingest %.1f ms, chain %.1f ms, file %.1f ms (%llu rows)\n", ms(t0, t1),
                    ms(t1, t2), ms(t2, clk::now()), (unsigned long long)m);
        }
    });
}

int st_compressed_ply_file(st_ctx *c, const st_ttable *src, const st_action *actions, int32_t nactions, int32_t out_fd,
                           const char *version, uint64_t *out_m, int32_t *out_sh_coeffs, uint64_t *size) {
    return guard([&] {
        ST_REQUIRE(c && src && out_m && out_sh_coeffs && size && (actions || nactions == 0), ST_ERR_ARG,
                   "NULL argument");
        check_src(src);
        sog_file_check(out_fd);
        use_device(c);
        Chain ch{c};
        upload_chain(c, src, ch);
        run_actions(ch, actions, nactions);
        const uint64_t m = ch.n, nch = (m + 255) / 256;
        auto *dchunk = wsT<float>(c, "chain.chunk", nch * 18);
        auto *dvert = wsT<uint32_t>(c, "chain.vert", m * 4);
        auto *dsh = wsT<uint8_t>(c, "chain.sh", m * 3 * (uint64_t)band_coeffs(ch.cols) + 1);
        int32_t C = 0;
        compressed_tail(ch, dchunk, dvert, dsh, &C);
        *size = compressed_ply_to_file(c, m, C, dchunk, dvert, dsh, out_fd, version);
        *out_m = m;
        *out_sh_coeffs = C;
    });
}

int st_ply_sog_bundle(st_ctx *c, int32_t fd, const st_ply_header *h, int32_t element, const st_action *actions,
                      int32_t nactions, int32_t iters, const double *draws, uint64_t ndraws, uint64_t *used,
                      uint16_t dos_time, uint16_t dos_date, uint8_t **out, uint64_t *out_size) {
    return sog_chain(
        c, [&](Chain &ch) {
            ST_REQUIRE(c && h && fd >= 0, ST_ERR_ARG, "NULL argument");
            ply_chain(c, fd, h, element, ch);
        },
        actions, nactions, iters, draws, ndraws, used, dos_time, dos_date, out, out_size, nullptr, nullptr);
}

int st_sog_bundle_process(st_ctx *c, const st_ttable *src, const st_action *actions, int32_t nactions, int32_t iters,
                          const double *draws, uint64_t ndraws, uint64_t *used, uint16_t dos_time, uint16_t dos_date,
                          uint8_t **out, uint64_t *out_size) {
    return sog_chain(
        c, [&](Chain &ch) {
            ST_REQUIRE(c && src, ST_ERR_ARG, "NULL argument");
            check_src(src);
            upload_chain(c, src, ch);
        },
        actions, nactions, iters, draws, ndraws, used, dos_time, dos_date, out, out_size, nullptr, nullptr);
}

int st_sog_process(st_ctx *c, const st_ttable *src, const st_action *actions, int32_t nactions, int32_t iters,
                   const double *draws, uint64_t ndraws, uint64_t *used, st_sog_meta *meta,
                   const st_sog_textures *out) {
    ST_REQUIRE_RC(meta && out, "NULL argument");
    return sog_chain(
        c, [&](Chain &ch) {
            ST_REQUIRE(c && src, ST_ERR_ARG, "NULL argument");
            check_src(src);
            upload_chain(c, src, ch);
        },
        actions, nactions, iters, draws, ndraws, used, 0, 0, nullptr, nullptr, meta, out);
}

int st_dev_sog_t(st_ctx *c, const st_ttable *t, int32_t iters, const double *draws, uint64_t ndraws, uint64_t *used,
                 st_sog_meta *meta, const st_sog_textures *out) {
    return guard([&] {
        ST_REQUIRE(c && t && meta && out, ST_ERR_ARG, "NULL argument");
        check_src(t);
        use_device(c);
        const uint64_t u = sog_tdev(c, t, iters, draws, ndraws, meta, out);
        if (used) *used = u;
    });
}

}  // extern "C"
