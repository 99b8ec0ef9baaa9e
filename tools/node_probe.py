#!/usr/bin/env python3
"""Where the Node drop-in's PLY -> .sog job spends its time (tools/bench_node.js on a 10M SH-3
binary PLY): the same run with ST_XFER_PRINT=1 (rate of every staged host copy) and ST_DEBUG's
streamed-file phase stamps on stderr."""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PLY = (['x', 'y', 'z', 'nx', 'ny', 'nz', 'f_dc_0', 'f_dc_1', 'f_dc_2'] + [f'f_rest_{i}' for i in range(45)] +
       ['opacity', 'scale_0', 'scale_1', 'scale_2', 'rot_0', 'rot_1', 'rot_2', 'rot_3'])
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
d = tempfile.mkdtemp(dir=os.environ.get('TMPDIR', '/tmp'))
src, dst = os.path.join(d, 'in.ply'), os.path.join(d, 'out.sog')
rng = np.random.default_rng(1002)
with open(src, 'wb') as f:
    f.write(('ply\nformat binary_little_endian 1.0\n' + f'element vertex {n}\n' +
             ''.join(f'property float {k}\n' for k in PLY) + 'end_header\n').encode())
    for a in range(0, n, 1 << 20):
        m = min(n, a + (1 << 20)) - a
        rows = rng.normal(0, 0.1, (m, len(PLY))).astype(np.float32)
        rows[:, 3:6] = 0
        f.write(rows.tobytes())
env = dict(os.environ, ST_XFER_PRINT='1', ST_DEBUG='1')
r = subprocess.run(['node', '--expose-gc', os.path.join(ROOT, 'tools', 'bench_node.js'), src, dst, '4', '10'], capture_output=True,
                   text=True, env=env, timeout=600)
print(r.stdout)
print('\n'.join(ln for ln in r.stderr.splitlines() if ln.startswith(('[st xfer]', '[st sog file]', '[addon]'))))
for p in (src, dst):
    if os.path.exists(p):
        os.remove(p)
os.rmdir(d)
sys.exit(r.returncode)
