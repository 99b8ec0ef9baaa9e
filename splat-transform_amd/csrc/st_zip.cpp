// st_zip.cpp -- the .sog container on the host: meta.json text and the store-only
// ZIP layout.  Byte-level parity with the reference is pinned
// by tests/golden/sog_bundle.* (the reference's own writeSog -> .sog with a pinned
// clock).
//
//   js_number      Number::toString as JSON.stringify emits it (ECMA-262 7.1.12.1:
//                  shortest round-trip digits, exponent form outside [1e-6, 1e21))
//   sog_meta_json  write-sog.ts:271-293 (means/scales/quats/sh0), :350-358 (shN), :361
//   zip_write      serialize/zip-writer.ts:35-135 (flags 0x808: CRC and sizes in a data
//                  descriptor after the data; method 0; DOS time/date of the writer's
//                  construction; central directory; end record without zip64)
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "st_webp.h"

namespace st {

std::string js_number(double v) {
    if (!std::isfinite(v)) return "null";
    if (v == 0) return "0";  // also -0
    std::string sign = v < 0 ? "-" : "";
    const double a = std::fabs(v);
    // shortest digit string that reads back as v (the correctly rounded p-digit decimal
    // is the closest one; its neighbours cover the asymmetric interval at powers of two)
    char buf[64];
    std::string digits;
    int exp10 = 0;
    for (int p = 1; p <= 17 && digits.empty(); ++p) {
        std::snprintf(buf, sizeof buf, "%.*e", p - 1, a);
        if (std::strtod(buf, nullptr) == a) {
            const char *e = std::strchr(buf, 'e');
            for (const char *q = buf; q < e; ++q)
                if (*q != '.') digits.push_back(*q);
            exp10 = std::atoi(e + 1);
        } else if (p < 17) {
            // try the neighbours of the rounded mantissa in the last place
            const char *e = std::strchr(buf, 'e');
            std::string m;
            for (const char *q = buf; q < e; ++q)
                if (*q != '.') m.push_back(*q);
            const int ex = std::atoi(e + 1);
            for (int dlt = -1; dlt <= 1 && digits.empty(); dlt += 2) {
                long long mv = std::atoll(m.c_str()) + dlt;
                if (mv <= 0) continue;
                std::string ms = std::to_string(mv);
                int ex2 = ex + (int)ms.size() - (int)m.size();
                std::snprintf(buf, sizeof buf, "%se%d", ms.c_str(), ex2 - (int)ms.size() + 1);
                if (std::strtod(buf, nullptr) == a) {
                    digits = ms;
                    exp10 = ex2;
                }
            }
        }
    }
    while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
    const int k = (int)digits.size();
    const int n = exp10 + 1;  // value = 0.d1d2...dk * 10^n
    std::string out;
    if (k <= n && n <= 21) {
        out = digits + std::string(n - k, '0');
    } else if (0 < n && n <= 21) {
        out = digits.substr(0, n) + "." + digits.substr(n);
    } else if (-6 < n && n <= 0) {
        out = "0." + std::string(-n, '0') + digits;
    } else {
        const int e = n - 1;
        out = digits.substr(0, 1);
        if (k > 1) out += "." + digits.substr(1);
        out += e >= 0 ? "e+" : "e-";
        out += std::to_string(e >= 0 ? e : -e);
    }
    return sign + out;
}

static std::string num_array(const float *v, int n) {
    std::string s = "[";
    for (int i = 0; i < n; ++i) {
        if (i) s += ",";
        s += js_number((double)v[i]);
    }
    return s + "]";
}

static std::string num_array(const double *v, int n) {
    std::string s = "[";
    for (int i = 0; i < n; ++i) {
        if (i) s += ",";
        s += js_number(v[i]);
    }
    return s + "]";
}

std::string sog_meta_json(const st_sog_meta &m, uint64_t count) {
    std::string s = "{\"version\":2,\"count\":" + std::to_string(count);
    s += ",\"means\":{\"mins\":" + num_array(m.means_min, 3) + ",\"maxs\":" + num_array(m.means_max, 3) +
         ",\"files\":[\"means_l.webp\",\"means_u.webp\"]}";
    s += ",\"scales\":{\"codebook\":" + num_array(m.scales_codebook, 256) + ",\"files\":[\"scales.webp\"]}";
    s += ",\"quats\":{\"files\":[\"quats.webp\"]}";
    s += ",\"sh0\":{\"codebook\":" + num_array(m.sh0_codebook, 256) + ",\"files\":[\"sh0.webp\"]}";
    if (m.sh_bands > 0) {
        s += ",\"shN\":{\"count\":" + std::to_string(m.palette_size) + ",\"bands\":" + std::to_string(m.sh_bands) +
             ",\"codebook\":" + num_array(m.shn_codebook, 256) +
             ",\"files\":[\"shN_centroids.webp\",\"shN_labels.webp\"]}";
    }
    return s + "}";
}

static inline void le16(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)v;
    p[1] = (uint8_t)(v >> 8);
}
static inline void le32(uint8_t *p, uint32_t v) {
    for (int k = 0; k < 4; ++k) p[k] = (uint8_t)(v >> (8 * k));
}

uint64_t zip_size(const std::vector<ZipEntry> &entries) {
    uint64_t s = 22;
    for (auto &e : entries) s += 30 + e.name.size() + e.size + 16 + 46 + e.name.size();
    return s;
}

size_t zip_local(const ZipEntry &e, uint16_t dos_time, uint16_t dos_date, uint8_t *h) {
    const uint32_t nl = (uint32_t)e.name.size();
    std::memset(h, 0, 30);
    le32(h + 0, 0x04034b50u);
    le16(h + 4, 20);            // version needed: 2.0
    le16(h + 6, 0x8 | 0x800);   // CRC/sizes in the descriptor, UTF-8 names
    le16(h + 8, 0);             // stored
    le16(h + 10, dos_time);
    le16(h + 12, dos_date);
    le16(h + 26, nl);
    std::memcpy(h + 30, e.name.data(), nl);
    return 30 + nl;
}

void zip_descriptor(const ZipEntry &e, uint8_t *d) {
    le32(d + 0, 0x08074b50u);
    le32(d + 4, e.crc);
    le32(d + 8, (uint32_t)e.size);
    le32(d + 12, (uint32_t)e.size);
}

uint64_t zip_central_size(const std::vector<ZipEntry> &entries) {
    uint64_t s = 22;
    for (auto &e : entries) s += 46 + e.name.size();
    return s;
}

void zip_central(const std::vector<ZipEntry> &entries, uint16_t dos_time, uint16_t dos_date, uint8_t *buf) {
    uint64_t o = 0, hdr = 0, names = 0, data = 0;
    for (size_t i = 0; i < entries.size(); ++i) {
        const ZipEntry &e = entries[i];
        const uint32_t nl = (uint32_t)e.name.size();
        uint8_t *c = buf + o;
        std::memset(c, 0, 46);
        le32(c + 0, 0x02014b50u);
        le16(c + 4, 20);
        le16(c + 6, 20);
        le16(c + 8, 0x8 | 0x800);
        le16(c + 10, 0);
        le16(c + 12, dos_time);
        le16(c + 14, dos_date);
        le32(c + 16, e.crc);
        le32(c + 20, (uint32_t)e.size);
        le32(c + 24, (uint32_t)e.size);
        le16(c + 28, nl);
        le32(c + 42, (uint32_t)hdr);  // the entry's local header: entries are laid out in order
        std::memcpy(c + 46, e.name.data(), nl);
        o += 46 + nl;
        hdr += 30 + nl + e.size + 16;
        names += nl;
        data += e.size;
    }
    uint8_t *z = buf + o;
    std::memset(z, 0, 22);
    const uint32_t n = (uint32_t)entries.size();
    le32(z + 0, 0x06054b50u);
    le16(z + 8, n);
    le16(z + 10, n);
    le32(z + 12, (uint32_t)(names + n * 46));
    le32(z + 16, (uint32_t)(names + n * (30 + 16) + data));
}

void zip_write(const std::vector<ZipEntry> &entries, uint16_t dos_time, uint16_t dos_date, uint8_t *buf,
               uint64_t *data_off) {
    uint64_t o = 0;
    for (size_t i = 0; i < entries.size(); ++i) {
        const ZipEntry &e = entries[i];
        o += zip_local(e, dos_time, dos_date, buf + o);
        data_off[i] = o;
        o += e.size;
        zip_descriptor(e, buf + o);
        o += 16;
    }
    zip_central(entries, dos_time, dos_date, buf + o);
}

}  // namespace st

using namespace st;

extern "C" {

void st_free(void *p) { std::free(p); }

int st_zip_store(const char *const *names, const uint8_t *const *data, const uint64_t *sizes, const uint32_t *crcs,
                 int32_t count, uint16_t dos_time, uint16_t dos_date, uint8_t **out, uint64_t *out_size) {
    return guard([&] {
        ST_REQUIRE(names && data && sizes && crcs && out && out_size && count >= 0, ST_ERR_ARG, "NULL argument");
        std::vector<ZipEntry> es;
        for (int i = 0; i < count; ++i) es.push_back({names[i], sizes[i], crcs[i]});
        const uint64_t total = zip_size(es);
        ST_REQUIRE(total < (1ull << 32), ST_ERR_ARG, "zip: archive exceeds 4 GiB (no zip64, as the reference)");
        uint8_t *buf = (uint8_t *)std::malloc(total);
        ST_REQUIRE(buf, ST_ERR_NOMEM, "zip: host allocation failed");
        std::vector<uint64_t> off(es.size());
        zip_write(es, dos_time, dos_date, buf, off.data());
        for (int i = 0; i < count; ++i)
            if (sizes[i]) std::memcpy(buf + off[i], data[i], sizes[i]);
        *out = buf;
        *out_size = total;
    });
}

int st_sog_meta_json(const st_sog_meta *meta, uint64_t count, char **out, uint64_t *out_size) {
    return guard([&] {
        ST_REQUIRE(meta && out && out_size, ST_ERR_ARG, "NULL argument");
        const std::string s = sog_meta_json(*meta, count);
        char *buf = (char *)std::malloc(s.size() + 1);
        ST_REQUIRE(buf, ST_ERR_NOMEM, "meta: host allocation failed");
        std::memcpy(buf, s.c_str(), s.size() + 1);
        *out = buf;
        *out_size = s.size();
    });
}

}  // extern "C"
