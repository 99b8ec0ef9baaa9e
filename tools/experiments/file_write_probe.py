#!/usr/bin/env python3
"""How fast can the box write a 158 MB .sog archive (the end-to-end leg's last step)?  The
archive sits in pinned host memory; written to TMPDIR by (a) one write(2), (b) 8 MiB write(2)s,
(c) O_DIRECT of the 4 KiB-aligned body + a buffered tail, (d) one write(2) into a file
preallocated with posix_fallocate (allocation outside the timed region).  Each form 3 times."""
import ctypes
import mmap
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, 'splat-transform_amd', 'py'))

size = 157_567_812
buf = mmap.mmap(-1, (size + 4095) // 4096 * 4096)  # page-aligned, like the pinned archive
buf.write(os.urandom(1 << 20) * (len(buf) >> 20))
addr = ctypes.addressof(ctypes.c_char.from_buffer(buf))
mv = memoryview(buf)[:size]
d = tempfile.mkdtemp(dir=os.environ.get('TMPDIR', '/tmp'))
path = os.path.join(d, 'out.sog')
print('TMPDIR', d, os.statvfs(d).f_bsize, flush=True)


def timed(name, fn, prep=None):
    ts = []
    for _ in range(3):
        if os.path.exists(path):
            os.remove(path)
        if prep:
            prep()
        t0 = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t0) * 1e3)
        assert os.path.getsize(path) == size
    print(f'{name:40s} {min(ts):7.1f} ms (min of 3; all {[round(t, 1) for t in ts]})', flush=True)


def one_write():
    with open(path, 'wb') as f:
        f.write(mv)


def chunked():
    with open(path, 'wb') as f:
        for o in range(0, size, 8 << 20):
            f.write(mv[o:o + (8 << 20)])


def direct():
    body = size // 4096 * 4096
    fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC | getattr(os, 'O_DIRECT', 0), 0o644)
    try:
        os.write(fd, memoryview(buf)[:body])
    finally:
        os.close(fd)
    with open(path, 'r+b') as f:
        f.seek(body)
        f.write(mv[body:])


def prealloc():
    fd = os.open(path, os.O_WRONLY | os.O_CREAT, 0o644)
    os.posix_fallocate(fd, 0, size)
    os.close(fd)


def into_prealloc():
    fd = os.open(path, os.O_WRONLY, 0o644)
    try:
        os.write(fd, mv)
    finally:
        os.close(fd)


timed('one write(2)', one_write)
timed('8 MiB write(2)s', chunked)
try:
    timed('O_DIRECT body + buffered tail', direct)
except OSError as e:
    print('O_DIRECT refused:', e)
timed('one write(2) into a preallocated file', into_prealloc, prealloc)
os.remove(path)
os.rmdir(d)
