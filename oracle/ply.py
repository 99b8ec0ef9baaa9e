"""CPU restatement of the PLY reader -- TEST INFRASTRUCTURE ONLY.

Checker for the product's PLY ingest (st_ply.hip).  Only tests/ import this
module.  Pinned by tests/golden/ply_io.* (the reference's readPly on a
mixed-type two-element file).

  read_ply   readers/read-ply.ts:111-191 (header search :114-137, parseHeader
             :54-110, the per-element row -> column copy :142-188)
"""
import numpy as np

TYPES = {'char': 'i1', 'uchar': 'u1', 'short': '<i2', 'ushort': '<u2', 'int': '<i4', 'uint': '<u4',
         'float': '<f4', 'double': '<f8'}
MAGIC = b'ply\n'
END = b'\nend_header\n'


class PlyError(ValueError):
    pass


def _parse_int(s):
    """JS parseInt(s, 10): leading whitespace, sign, digits; NaN -> None"""
    s = s.lstrip(' \t\n\r\v\f')
    i = 0
    sign = 1
    if i < len(s) and s[i] in '+-':
        sign = -1 if s[i] == '-' else 1
        i += 1
    j = i
    while j < len(s) and s[j].isdigit():
        j += 1
    return sign * int(s[i:j]) if j > i else None


def header_size(data):
    if len(data) < 16 or data[:4] != MAGIC:
        raise PlyError('invalid file header' if len(data) >= 16 else 'failed to read file header')
    # the reader grows the header one byte at a time from 16 bytes and checks whether it ends
    # with "\nend_header\n" (read-ply.ts:126-137); at most 128 KiB
    k = data.find(END, 5)
    if k < 0 or k + len(END) > 128 * 1024:
        raise PlyError('failed to read file header')
    return k + len(END)


def parse_header(text):
    """read-ply.ts:54-110 -> (comments, [(name, count, [(prop, type)])])"""
    lines = [ln for ln in text.split('\n') if ln]
    comments, elements = [], []
    for line in lines[1:]:
        words = line.split(' ')
        w0 = words[0]
        if w0 in ('ply', 'format', 'end_header'):
            continue
        if w0 == 'comment':
            comments.append(line[8:])
        elif w0 == 'element':
            if len(words) != 3:
                raise PlyError('invalid ply header')
            cnt = _parse_int(words[2])
            if cnt is not None and cnt < 0:
                raise PlyError('invalid typed array length')
            elements.append((words[1], cnt or 0, []))
        elif w0 == 'property':
            if not elements or len(words) != 3 or words[1] not in TYPES:
                raise PlyError('invalid ply header')
            elements[-1][2].append((words[2], words[1]))
        else:
            raise PlyError(f"unrecognized header value '{w0}' in ply header")
    return comments, elements


def read_ply(data):
    """-> (comments, [(name, {prop: array})]) with columns in property order"""
    data = bytes(data)
    hs = header_size(data)
    comments, elements = parse_header(data[:hs].decode('latin-1'))
    off = hs
    out = []
    for name, count, props in elements:
        dt = np.dtype([(f'p{i}', TYPES[t]) for i, (_, t) in enumerate(props)]) if props else None
        cols = {}
        if dt is not None and count:
            need = count * dt.itemsize
            if off + need > len(data):
                raise PlyError('file shorter than its header declares')
            rows = np.frombuffer(data, dtype=dt, count=count, offset=off)
            for i, (pn, _) in enumerate(props):
                cols[pn] = rows[f'p{i}'].astype(TYPES[props[i][1]]).copy()
            off += need
        else:
            for pn, t in props:
                cols[pn] = np.zeros(0, TYPES[t])
        out.append((name, cols))
    return comments, out
