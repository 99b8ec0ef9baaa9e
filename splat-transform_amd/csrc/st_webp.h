// st_webp.h -- device WebP lossless encode, CRC-32, and the SOG container (internal).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "st_internal.h"

namespace st {

struct WebpJob {
    const uint8_t *rgba;  // device, RGBA8 rows
    int w, h, stride;     // stride in bytes (multiple of 4)
    uint8_t *out;         // device, >= webp_max_size(w, h) bytes, 4-byte aligned
    uint64_t cap;
    uint64_t size;        // out: bytes of the .webp file
    bool cache = true;    // try a colour cache (the hit search costs ~0.6 ms per 10 MPix image)
};
// the .sog textures a colour cache pays for: measured at 10M SH-3 (profiles/r05/colour_cache.json),
// only the means textures gain (means_l -0.36%, means_u -2.3%); the others gain bytes, not percents
bool sog_texture_cache(const char *name);

uint64_t webp_max_size(int w, int h);
// encodes every job (three stream synchronisations for the whole batch)
void webp_encode_dev(st_ctx *c, WebpJob *jobs, int njobs);
// zlib-compatible CRC-32 of cnt device buffers (crc_in: running value, 0 for a fresh CRC)
void crc32_dev(st_ctx *c, const uint8_t *const *data, const uint64_t *n, const uint32_t *crc_in, int cnt,
               uint32_t *crcs);

// the whole .sog archive (WebP-encoded textures + meta.json, zip-writer.ts layout) of
// textures resident on the device, in the context's pinned archive buffer (valid until
// the next bundle call on this context)
void sog_bundle_dev(st_ctx *c, const st_sog_meta &meta, uint64_t count, const st_sog_textures &tex,
                    uint16_t dos_time, uint16_t dos_date, const uint8_t **out, uint64_t *out_size);
// writeSog into an open file: the step (sog_dev) with the archive streamed to fd -- the five
// textures final before the SH k-means encoded on the side context and written by a host thread
// while the k-means runs; the same bytes as sog_bundle_dev's archive.  Returns the draws used.
uint64_t sog_file_dev(st_ctx *c, const st_table *t, int iters, const double *draws, uint64_t ndraws,
                      st_sog_meta *meta, const st_sog_textures *out, int fd, uint16_t dos_time, uint16_t dos_date,
                      uint64_t *file_size);
// the descriptor checks of the file writers: fd must be a seekable file (ST_ERR_ARG otherwise);
// write n bytes at offset off; cut a longer file to `size` bytes
void sog_file_check(int fd);
void write_at(int fd, const uint8_t *p, uint64_t n, uint64_t off);
void sog_file_truncate(int fd, uint64_t size);

// ---- host: the .sog container (st_zip.cpp) ----------------------------------
// JSON text of a JS number (Number::toString as JSON.stringify emits it; non-finite -> null)
std::string js_number(double v);
// meta.json of writeSog (write-sog.ts:271-293, 350-361)
std::string sog_meta_json(const st_sog_meta &m, uint64_t count);

struct ZipEntry {
    std::string name;
    uint64_t size;
    uint32_t crc;
};
// the store-only archive of serialize/zip-writer.ts: per entry a local header, the
// data and a data descriptor; then the central directory and the end record.
uint64_t zip_size(const std::vector<ZipEntry> &entries);
// writes everything but the entries' data into buf (zip_size bytes); data_off[i] = where
// entry i's bytes go
void zip_write(const std::vector<ZipEntry> &entries, uint16_t dos_time, uint16_t dos_date, uint8_t *buf,
               uint64_t *data_off);
// the pieces zip_write lays out, for a writer that streams the entries: one entry's local header
// (returns its 30 + name bytes; independent of the entry's size and CRC), its 16-byte data
// descriptor, and the central directory + end record of entries laid out in order from offset 0
size_t zip_local(const ZipEntry &e, uint16_t dos_time, uint16_t dos_date, uint8_t *h);
void zip_descriptor(const ZipEntry &e, uint8_t *d);
uint64_t zip_central_size(const std::vector<ZipEntry> &entries);
void zip_central(const std::vector<ZipEntry> &entries, uint16_t dos_time, uint16_t dos_date, uint8_t *buf);

}  // namespace st
