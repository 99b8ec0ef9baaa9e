"""CPU restatement of the .sog container -- TEST INFRASTRUCTURE ONLY.

Checker for the product's WebP/CRC/ZIP/meta path (st_webp.hip, st_zip.cpp).
Only tests/ import this module.  Pinned by tests/golden/sog_bundle.* (the
reference's writeSog -> .sog run with a fixed clock, tests/golden/gen/make_golden.js).

  crc32          serialize/crc.ts:1-28 (table-driven, init -1, final xor -1)
  zip_store      serialize/zip-writer.ts:35-135
  js_number      ECMA-262 Number::toString (what JSON.stringify emits for numbers)
  sog_meta_json  write-sog.ts:271-293, :350-361
"""
import struct


def _crc_table():
    # crc.ts:1-13
    tbl = []
    for n in range(256):
        c = n
        for _ in range(8):
            c = (0xEDB88320 ^ (c >> 1)) if (c & 1) else (c >> 1)
        tbl.append(c)
    return tbl


_TBL = _crc_table()


def crc32(data, crc=0):
    """crc.ts:15-28: bits = -1; bits = (bits >>> 8) ^ table[(bits ^ byte) & 0xff]; value = bits ^ -1"""
    bits = crc ^ 0xFFFFFFFF
    for b in bytes(data):
        bits = (bits >> 8) ^ _TBL[(bits ^ b) & 0xFF]
    return bits ^ 0xFFFFFFFF


def dos_clock(year, month0, day, hours, minutes, seconds):
    """zip-writer.ts:39-41 (month0 as JS Date's 0-based month)"""
    dos_time = (hours << 11) | (minutes << 5) | (seconds // 2)
    dos_date = ((year - 1980) << 9) | ((month0 + 1) << 5) | day
    return dos_time, dos_date


def zip_store(entries, dos_time, dos_date):
    """entries: [(name, bytes)] in write order; the archive bytes of ZipWriter.file()* + close()"""
    out = bytearray()
    files = []
    for name, data in entries:
        fn = name.encode('utf-8')
        # writeHeader (zip-writer.ts:43-62): 30-byte local header, sizes/crc zero
        hdr = bytearray(30)
        struct.pack_into('<IHHHHH', hdr, 0, 0x04034b50, 20, 0x8 | 0x800, 0, dos_time, dos_date)
        struct.pack_into('<H', hdr, 26, len(fn))
        out += hdr + fn
        out += bytes(data)
        c = crc32(data)
        # writeFooter (zip-writer.ts:64-74): data descriptor
        out += struct.pack('<IIII', 0x08074b50, c, len(data), len(data))
        files.append((fn, c, len(data)))
    # close (zip-writer.ts:90-132): central directory + end record
    offset = 0
    for fn, c, size in files:
        cdr = bytearray(46)
        struct.pack_into('<IHHHHHHIII', cdr, 0, 0x02014b50, 20, 20, 0x8 | 0x800, 0, dos_time, dos_date, c, size,
                         size)
        struct.pack_into('<H', cdr, 28, len(fn))
        struct.pack_into('<I', cdr, 42, offset)
        out += cdr + fn
        offset += 30 + len(fn) + size + 16
    name_len = sum(len(f[0]) for f in files)
    data_len = sum(f[2] for f in files)
    eocd = bytearray(22)
    struct.pack_into('<I', eocd, 0, 0x06054b50)
    struct.pack_into('<HH', eocd, 8, len(files), len(files))
    struct.pack_into('<I', eocd, 12, name_len + len(files) * 46)
    struct.pack_into('<I', eocd, 16, name_len + len(files) * (30 + 16) + data_len)
    out += eocd
    return bytes(out)


def js_number(v):
    """Number::toString(v) for finite v (JSON.stringify: non-finite -> null, -0 -> 0)"""
    v = float(v)
    if v != v or v in (float('inf'), float('-inf')):
        return 'null'
    if v == 0:
        return '0'
    sign = '-' if v < 0 else ''
    # repr gives the shortest round-trip digits (the ECMAScript digit choice)
    r = repr(abs(v))
    if 'e' in r:
        mant, e = r.split('e')
        exp = int(e)
    else:
        mant, exp = r, 0
    if '.' in mant:
        ip, fp = mant.split('.')
    else:
        ip, fp = mant, ''
    digits = (ip + fp).lstrip('0')
    lead_zeros = len(ip + fp) - len((ip + fp).lstrip('0'))
    n = len(ip) + exp - lead_zeros  # decimal point position relative to the first significant digit
    digits = digits.rstrip('0') or '0'
    k = len(digits)
    if k <= n <= 21:
        s = digits + '0' * (n - k)
    elif 0 < n <= 21:
        s = digits[:n] + '.' + digits[n:]
    elif -6 < n <= 0:
        s = '0.' + '0' * (-n) + digits
    else:
        e = n - 1
        s = digits[0] + ('.' + digits[1:] if k > 1 else '') + ('e+' if e >= 0 else 'e-') + str(abs(e))
    return sign + s


def _arr(vals):
    return '[' + ','.join(js_number(x) for x in vals) + ']'


def sog_meta_json(count, means_min, means_max, scales_codebook, sh0_codebook, sh_bands=0, palette_size=0,
                  shn_codebook=None):
    """JSON.stringify(meta) of write-sog.ts:271-293 (+ shN, :350-358); float32 codebooks as their f64 values"""
    s = '{"version":2,"count":%d' % count
    s += ',"means":{"mins":%s,"maxs":%s,"files":["means_l.webp","means_u.webp"]}' % (_arr(means_min),
                                                                                       _arr(means_max))
    s += ',"scales":{"codebook":%s,"files":["scales.webp"]}' % _arr(scales_codebook)
    s += ',"quats":{"files":["quats.webp"]}'
    s += ',"sh0":{"codebook":%s,"files":["sh0.webp"]}' % _arr(sh0_codebook)
    if sh_bands > 0:
        s += (',"shN":{"count":%d,"bands":%d,"codebook":%s,"files":["shN_centroids.webp","shN_labels.webp"]}'
              % (palette_size, sh_bands, _arr(shn_codebook)))
    return (s + '}').encode()
