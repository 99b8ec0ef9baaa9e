"""PLY ingest and the compressed-PLY reader on the host side (no GPU): the oracle
restatements against the reference's own outputs (tests/golden/ply_io.*: readPly on a
mixed-type two-element file, decompressPly of the compressed_ply fixture files), and
the product's header parser (st_ply_parse_header) against the oracle, errors included.
"""
import numpy as np
import pytest

import oracle
import ply
import splat_hip as sh
from golden_io import Golden

G = Golden('ply_io')
CP = Golden('compressed_ply')


def compressed_file(name):
    return b''.join(CP[f'{name}_{k}'].tobytes() for k in ('header', 'chunk', 'vertex', 'sh'))


def same(a, b):
    return a.dtype.itemsize == b.dtype.itemsize and np.array_equal(a.view(f'u{a.dtype.itemsize}'),
                                                                    b.view(f'u{b.dtype.itemsize}'))


def test_oracle_read_ply_matches_reference():
    comments, els = ply.read_ply(G['mixed_file'].tobytes())
    assert comments == G.meta['mixed']['comments']
    assert [(n, list(c)) for n, c in els] == [(e['name'], [k for k, _ in e['columns']])
                                             for e in G.meta['mixed']['elements']]
    for name, cols in els:
        for k, v in cols.items():
            assert same(v, G[f'mixed_{name}_{k}']), (name, k)


@pytest.mark.parametrize('name', [c['name'] for c in G.meta['compressed']])
def test_oracle_decompress_matches_reference(name):
    _, els = ply.read_ply(compressed_file(name))
    el = dict(els)
    shc = [el['sh'][f'f_rest_{i}'] for i in range(len(el['sh']))] if 'sh' in el else []
    out = oracle.decompress_ply(el['chunk'], el['vertex'], shc)
    assert list(out) == G.meta[f'{name}_columns']
    for k, v in out.items():
        assert same(v, G[f'{name}_dec_{k}']), k


def _headers():
    base = b'ply\nformat binary_little_endian 1.0\nelement vertex 3\nproperty float x\nend_header\n'
    return {
        'ok': base,
        'comments': b'ply\ncomment a b\ncomment\nelement v 2\nproperty uchar q\nproperty double w\nend_header\n',
        'two_elements': b'ply\nelement a 1\nproperty int i\nelement b 5\nproperty short s\nend_header\n',
        'nan_count': b'ply\nelement vertex abc\nproperty float x\nend_header\n',
        'count_suffix': b'ply\nelement vertex 12xyz\nproperty float x\nend_header\n',
        'bad_magic': b'plx\nelement vertex 3\nproperty float x\nend_header\n',
        'no_end': b'ply\nelement vertex 3\nproperty float x\n' + b' ' * 40,
        'short': b'ply\nend',
        'list_prop': b'ply\nelement face 1\nproperty list uchar int idx\nend_header\n',
        'bad_type': b'ply\nelement vertex 1\nproperty half x\nend_header\n',
        'prop_first': b'ply\nproperty float x\nelement vertex 1\nend_header\n',
        'unknown': b'ply\nobj_info foo\nelement vertex 1\nend_header\n',
        'two_spaces': b'ply\nelement  vertex 1\nend_header\n',
        'negative': b'ply\nelement vertex -2\nend_header\n',
    }


@pytest.mark.parametrize('kind', list(_headers().keys()))
def test_header_parser_matches_oracle(kind):
    data = _headers()[kind]
    try:
        hs = ply.header_size(data)
        want = ply.parse_header(data[:hs].decode('latin-1'))
        err = None
    except ply.PlyError as e:
        want, err = None, str(e)
    if err is None:
        h = sh.ply_parse_header(data)
        assert h.header_bytes == hs
        comments, elements = want
        assert h.comment_list() == comments
        got = [(n, c, [(p, np.dtype(t).str) for p, t in props]) for n, c, props in h.layout()]
        assert got == [(n, c, [(p, np.dtype(ply.TYPES[t]).str) for p, t in props]) for n, c, props in elements]
    else:
        with pytest.raises(sh.StError) as ei:
            sh.ply_parse_header(data)
        assert err in str(ei.value)


def test_header_of_fixture_files():
    h = sh.ply_parse_header(G['mixed_file'].tobytes())
    assert h.comment_list() == G.meta['mixed']['comments']
    for name in ('sh3', 'sh0'):
        f = compressed_file(name)
        assert sh.ply_parse_header(f).header_bytes == ply.header_size(f)
