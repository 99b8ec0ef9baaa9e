#!/usr/bin/env python3
"""Stage the reference's hot-path modules as runnable CommonJS in /tmp.

TEST INFRASTRUCTURE ONLY.  Reads /root/reference/src/*.ts (read-only), erases
TypeScript types with strip_ts.py and writes the result to
$ST_REF_JS (default /tmp/st_ref_js).  Nothing produced here is committed; only
the fixture vectors that make_golden.js derives from running it are.

Substitutions (all at module-import level, never inside a function body):
  * 'playcanvas'            -> pc_math.js, a restatement of playcanvas@2.11.8 math
  * '../utils/webp'         -> identity encoder: the reference's prebuilt
                               lib/webp_encode.wasm is never executed; WebP
                               lossless is decoded back to the same RGBA, so
                               fixtures record that RGBA instead
  * '../gpu/*'              -> throwing stubs (only the --no-gpu path is used)
  * node:* builtins         -> Node 12 equivalents
  * two test-only exports appended: `combine` (index.ts) and `cluster1d`
    (write-sog.ts), which the reference defines but does not export.
"""
import os
import re
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from strip_ts import strip, lower_modules, lower_nullish, tokenize  # noqa: E402

REF = os.environ.get('ST_REFERENCE', '/root/reference')
OUT = os.environ.get('ST_REF_JS', '/tmp/st_ref_js')

FILES = [
    'data-table', 'ordering', 'compressed-chunk', 'transform', 'process', 'index',
    'utils/math', 'utils/rotate-sh', 'utils/kd-tree', 'utils/k-means',
    'writers/write-compressed-ply', 'writers/write-sog',
    'serialize/crc', 'serialize/writer', 'serialize/zip-writer',
    'readers/read-ply', 'readers/decompress-ply',
]

EXTRA_EXPORTS = {
    'index': ['combine'],
    'writers/write-sog': ['cluster1d', 'generateIndices'],
}

STUBS = {
    '__stubs/fs_promises.js': "module.exports = require('fs').promises;\n",
    '__stubs/gpu_device.js': "module.exports = { createDevice: () => { throw new Error('gpu path not used in fixtures'); } };\n",
    '__stubs/gpu_clustering.js': "module.exports = { GpuClustering: function () { throw new Error('gpu path not used in fixtures'); } };\n",
    '__stubs/empty.js': "module.exports = {};\n",
    '__stubs/webp.js': (
        "// identity stand-in for the lossless WebP encoder: emits the raw RGBA\n"
        "// preceded by a 16-byte header (magic 'RGBA', width, height, byteLength).\n"
        "class WebpEncoder {\n"
        "    static async create() { return new WebpEncoder(); }\n"
        "    encodeLosslessRGBA(rgba, width, height) {\n"
        "        const out = Buffer.alloc(16 + rgba.length);\n"
        "        out.write('RGBA', 0, 'ascii');\n"
        "        out.writeUInt32LE(width, 4); out.writeUInt32LE(height, 8); out.writeUInt32LE(rgba.length, 12);\n"
        "        Buffer.from(rgba.buffer, rgba.byteOffset, rgba.length).copy(out, 16);\n"
        "        return out;\n"
        "    }\n"
        "}\n"
        "module.exports = { WebpEncoder };\n"),
}

INDEX_UNUSED = ['./readers/', './writers/write-csv', './writers/write-html', './writers/write-ply']


def make_resolver(rel):
    here = os.path.dirname(rel)

    def resolve(spec):
        if spec == 'playcanvas':
            return os.path.join(OUT, '__stubs/playcanvas.js')
        if spec == 'node:fs/promises':
            return os.path.join(OUT, '__stubs/fs_promises.js')
        if spec.startswith('node:'):
            return spec[5:]
        if spec.endswith('package.json'):
            return os.path.join(REF, 'package.json')
        if spec.startswith('.'):
            target = os.path.normpath(os.path.join(here, spec))
            if target.endswith('.js'):
                target = target[:-3]
            if target == 'utils/webp':
                return os.path.join(OUT, '__stubs/webp.js')
            if target == 'gpu/gpu-device':
                return os.path.join(OUT, '__stubs/gpu_device.js')
            if target == 'gpu/gpu-clustering':
                return os.path.join(OUT, '__stubs/gpu_clustering.js')
            if rel == 'index' and any(spec.startswith(p) for p in INDEX_UNUSED):
                return os.path.join(OUT, '__stubs/empty.js')
            return os.path.join(OUT, target + '.js')
        return spec
    return resolve


def lower_optchain(src):
    # `a?.b` -> `(a == null ? undefined : a.b)` for the simple identifier form
    return re.sub(r'\b(\w+)\?\.(\w+)', r'(\1 == null ? undefined : \1.\2)', src)


def main():
    if os.path.isdir(OUT):
        shutil.rmtree(OUT)
    os.makedirs(os.path.join(OUT, '__stubs'))
    for name, body in STUBS.items():
        with open(os.path.join(OUT, name), 'w') as f:
            f.write(body)
    shutil.copy(os.path.join(HERE, 'pc_math.js'), os.path.join(OUT, '__stubs/playcanvas.js'))
    for rel in FILES:
        src = open(os.path.join(REF, 'src', rel + '.ts')).read()
        # type-only imports have no runtime part
        src = re.sub(r'^import type [^;]*;\n', '', src, flags=re.M)
        # non-null assertions `x!.y`
        src = re.sub(r'([\w\)\]])!\.', r'\1.', src)
        js = strip(src)
        js = lower_modules(js, make_resolver(rel))
        js = lower_nullish(js)
        js = lower_optchain(js)
        extra = EXTRA_EXPORTS.get(rel)
        if extra:
            js += '\n' + ''.join(f'module.exports.{n} = {n};\n' for n in extra)
        js = ("'use strict';\n"
              "const __nc = (a, b) => (a !== null && a !== undefined ? a : b);\n" + js)
        dst = os.path.join(OUT, rel + '.js')
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        with open(dst, 'w') as f:
            f.write(js)
        # sanity: no TypeScript-only tokens survive
        for tk in tokenize(js):
            if tk.kind == 'ident' and tk.text in ('interface', 'private'):
                raise AssertionError(f'{rel}: leftover {tk.text}')
    print(OUT)


if __name__ == '__main__':
    main()
