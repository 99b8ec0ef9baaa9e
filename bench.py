#!/usr/bin/env python3
"""bench.py -- Msplats/s PLY->SOG (SH-3, 10 k-means iters) on MI355X.

One step = the whole SOG device pipeline of write-sog.ts:110-370 over a synthetic SH-3 splat
table already resident in HBM: Morton order, means / quats textures, cluster1d(scales),
cluster1d(f_dc) + opacity, the SH palette k-means (K = 65,536, 10 iterations), the codebook
cluster1d and the shN textures (the headline is the device pipeline).  The .sog
container stage -- WebP lossless encode of the seven textures, CRC-32 and the ZIP layout
(st_dev_sog_bundle_view, archive in pinned host memory) -- is timed right after on the same
textures and reported in "container" with the end-to-end rate.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--splats S] [--total-splats T] [--merge F]

Workloads (BASELINE.json configs):
  default (every N)     north_star's workload: ONE 10M-splat SH-3 table (seed 1002), strong-scaled
                        -- at N = 1 through st_dev_sog, at N > 1 split N ways by rows, each rank
                        running st_dev_sog_sharded (the library's RCCL exchange, st_multi.hip).
                        `config.workload` is the same string at every N.  Extra records beside
                        it: N = 1 `sharded_world1` (the same table through st_dev_sog_sharded
                        over a one-rank RCCL communicator: the sharded path's own denominator),
                        every N `config4_50M` (one 50M-splat table, strong) and, N > 1,
                        `weak_10M_per_gpu` (10M splats per GPU)
  --merge F             config 5: F input tables of 10M splats (--file-splats) concatenated
                        (combine, index.ts:158-210) + Morton + SOG, the rows split over the ranks
  --total-splats T      one T-splat table split over the ranks (strong)
  --splats S            S splats per GPU (weak)
N > 1 runs one process per GPU.  `python bench.py --gpus N` with no launcher around it starts
the N-rank job itself (a child `python -m torch.distributed.run --nproc-per-node N ...`, spawned
before this process touches torch or the GPU), relays rank 0's JSON line and fails unless the
job ran N ranks; under torchrun (WORLD_SIZE set) the ranks run directly.  torch.distributed
carries only the RCCL unique id, the barriers and the max-over-ranks timing.

Synthetic tables are built from fixed-seed blocks of 10M rows (block b: seed 1002 + b), and a
rank takes its global row range of them, so a T-splat table is the same table for every N (its
`textures_sha256` does not depend on N); 10M splats per GPU is block `rank`.

Prints ONE JSON line (rank 0) with the roofline of the dominant kernel (the MFMA assign
sweep, measured with HIP events on its own stream), the CPU-oracle baseline timed on a
bounded sample, and the verification of the last step's output.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, 'splat-transform_amd', 'py'))

MFMA_F16_DENSE_TFLOPS = 2500.0  # MI355X dense fp16/bf16 MFMA peak (MI355X_MICROARCH.md)
HBM_TBPS = 8.0


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--splats', type=int, default=None, help='splats per GPU (weak scaling; default 10M at N = 1)')
    ap.add_argument('--total-splats', type=int, default=None,
                    help='one table of this many splats split over the ranks (default 50M at N > 1: config 4)')
    ap.add_argument('--merge', type=int, default=0, help='config 5: this many input tables concatenated')
    ap.add_argument('--file-splats', type=int, default=10_000_000, help='rows per --merge input')
    ap.add_argument('--no-weak', '--no-extra', dest='no_extra', action='store_true',
                    help='skip the extra records (sharded_world1, config4_50M, weak_10M_per_gpu)')
    ap.add_argument('--extra-steps', type=int, default=3, help='timed steps of each extra record (1 warmup)')
    ap.add_argument('--iters', type=int, default=10, help='k-means iterations (reference default 10)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--backend', default='nccl', help='torch.distributed backend for N > 1 (nccl = RCCL; gloo with '
                    '--dist-python rehearses several ranks on one GPU)')
    ap.add_argument('--torch-backend', default='auto', choices=('auto', 'gloo', 'nccl'),
                    help='the process group of bench.py\'s own between-step duties (barriers, the unique id\'s '
                         'broadcast, the max-over-ranks timer, the verification\'s reductions); auto: gloo, except '
                         'nccl for --dist-python (its collectives are the step\'s), so that the library\'s RCCL is the '
                         'only one a rank initialises')
    ap.add_argument('--cpu-assign-sample', type=int, default=20_000,
                    help='points of the 1-thread KdTree assign sample (cpu_baseline)')
    ap.add_argument('--cpu-assign-sample-mt', type=int, default=100_000,
                    help='points of the all-cores assign sample (cpu_baseline_all_cores; BASELINE.md: 100k rows)')
    ap.add_argument('--cpu-rest-sample', type=int, default=200_000)
    ap.add_argument('--no-e2e', action='store_true', help='skip the PLY file -> .sog file measurement (N = 1)')
    ap.add_argument('--no-paths', action='store_true', help='skip the config-3 stage table (N = 1)')
    ap.add_argument('--no-verify', action='store_true', help='skip the output verification of the last step')
    ap.add_argument('--verify-sample', action='store_true',
                    help='verify 4,096 sampled labels instead of every label of the last assign')
    ap.add_argument('--dist', action='store_true', help='N = 1 through the sharded code path (st_dev_sog_sharded '
                    'over a one-rank RCCL communicator) instead of st_dev_sog: its per-rank cost')
    ap.add_argument('--dist-python', action='store_true', help='the sharded path through splat_dist.py '
                    '(torch.distributed collectives around the step API) instead of the library')
    ap.add_argument('--launch-dry-run', action='store_true', help=argparse.SUPPRESS)  # print the launcher command
    ap.add_argument('--launch-budget', type=float, default=1500.0,
                    help='self-launched N-rank job: seconds before it is killed (then rerun once with the side '
                         'channel off)')
    ap.add_argument('--launch-stall', type=float, default=300.0,
                    help='self-launched N-rank job: seconds without a progress line from any rank before it is '
                         'killed (600 s before the first one: imports, RCCL set-up)')
    ap.add_argument('--rank-watchdog', type=float, default=900.0,
                    help='N > 1: a rank that makes no progress for this many seconds reports its phase and exits '
                         '(124), so a hung job ends with a diagnosis instead of at the driver\'s limit; 0 = off')
    return ap.parse_args(argv)


def launcher_cmd(argv, n, port):
    """the N-rank job `bench.py --gpus N` starts when no launcher is around it"""
    return [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={n}',
            '--master-addr=127.0.0.1', f'--master-port={port}', os.path.abspath(__file__)] + list(argv)


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def run_job(cmd, env, budget, stall, first_stall=600.0):
    """run the N-rank job, relaying its output; returns (exit code, result line or None, why it was
    stopped or None).  Ranks write '@@progress' lines to stdout (BENCH_PROGRESS=1); the job is
    killed (its whole process group) after `budget` seconds, or after `stall` seconds without a
    progress line (`first_stall` before the first one)."""
    import queue
    import signal
    import subprocess
    import threading
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, env=env, text=True, start_new_session=True)
    q = queue.Queue()

    def reader():
        for ln in proc.stdout:
            q.put(ln)
        q.put(None)
    threading.Thread(target=reader, daemon=True).start()
    t0 = time.time()
    last, seen, line, why = t0, False, None, None
    while True:
        try:
            ln = q.get(timeout=1.0)
        except queue.Empty:
            ln = ''
        now = time.time()
        if ln is None:
            break
        if ln.startswith('@@progress'):
            last, seen = now, True
            sys.stderr.write('bench.py: ' + ln[2:])
        elif ln.startswith('{') and '"metric"' in ln:
            line = ln.strip()
        elif ln:
            sys.stderr.write(ln)
        if now - t0 > budget:
            why = f'no result within the {budget:.0f} s budget'
        elif now - last > (stall if seen else first_stall):
            why = f'no progress line for {now - last:.0f} s'
        if why:
            print(f'bench.py: killing the job: {why}', file=sys.stderr, flush=True)
            for sig, wait in ((signal.SIGTERM, 15), (signal.SIGKILL, 30)):
                try:
                    os.killpg(proc.pid, sig)
                except ProcessLookupError:
                    break
                try:
                    proc.wait(timeout=wait)
                    break
                except subprocess.TimeoutExpired:
                    pass
            break
    rc = proc.wait()
    return rc, line, why


def launch(args, argv):
    """parent of a self-launched N-rank job: never imports torch (nothing here touches the GPU);
    the ranks' stdout is read here, rank 0's JSON line relayed, everything else goes to stderr.
    A job that stalls or fails is rerun once with the side channel off (ST_SIDE_CHANNEL=0: every
    exchange on the main communicator, in one host thread's program order) and the library's
    collectives on torch's RCCL (ST_RCCL=process), and the line says so."""
    cmd = launcher_cmd(argv, args.gpus, free_port())
    if args.launch_dry_run:
        _RESULT.write(json.dumps({'cmd': cmd, 'torch_imported': 'torch' in sys.modules}) + '\n')
        _RESULT.flush()
        return 0
    env = dict(os.environ)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    env.setdefault('OMP_NUM_THREADS', '1')
    env['BENCH_PROGRESS'] = '1'
    print('bench.py: launching ' + ' '.join(cmd), file=sys.stderr, flush=True)
    rc, line, why = run_job(cmd, env, args.launch_budget, args.launch_stall)
    fallback = None
    if line is None:
        first = why or f'exit code {rc}'
        print(f'bench.py: the {args.gpus}-rank job ended without a result ({first}); rerunning it once with the '
              'side channel off (ST_SIDE_CHANNEL=0)', file=sys.stderr, flush=True)
        env['ST_SIDE_CHANNEL'] = '0'
        # and the collectives on the RCCL torch already loaded (st_rccl.h: ST_RCCL=process) instead
        # of a second copy beside it
        env.setdefault('ST_RCCL', 'process')
        cmd = launcher_cmd(argv, args.gpus, free_port())
        rc, line, why = run_job(cmd, env, args.launch_budget, args.launch_stall)
        fallback = {'side_channel': 'off', 'rccl': env['ST_RCCL'], 'first_job': first}
    if line is None:
        print(f'bench.py: the {args.gpus}-rank job exited with {rc}' + (f' ({why})' if why else ''), file=sys.stderr)
        return rc or 3
    if rc != 0:
        print(f'bench.py: the {args.gpus}-rank job exited with {rc}', file=sys.stderr)
        return rc
    res = json.loads(line)
    if res.get('n_gpus') != args.gpus:
        print(f'bench.py: the job ran {res.get("n_gpus")} ranks, not {args.gpus}', file=sys.stderr)
        return 3
    if fallback:
        res['fallback'] = fallback
        line = json.dumps(res)
    _RESULT.write(line + '\n')
    _RESULT.flush()
    return 0


_LAST_PROGRESS = [0.0]


def progress(what):
    """a progress mark: a '@@progress' line for the self-launching parent's watchdog (only when it
    asked for them: stdout otherwise carries exactly the one JSON line) and the rank watchdog's
    clock"""
    _LAST_PROGRESS[0] = time.time()
    _PHASE[0] = what
    if os.environ.get('BENCH_PROGRESS') == '1':
        _RESULT.write(f'@@progress rank={os.environ.get("RANK", "0")} {what}\n')
        _RESULT.flush()


def rank_watchdog(limit):
    """N > 1: a rank whose progress marks stop for `limit` seconds (a hung collective) prints its
    phase and exits with 124; the launcher then ends the other ranks"""
    import threading
    if limit <= 0:
        return
    _LAST_PROGRESS[0] = time.time()

    def run():
        while True:
            time.sleep(5)
            idle = time.time() - _LAST_PROGRESS[0]
            if idle > limit:
                print(f'bench.py: rank {os.environ.get("RANK", "0")} made no progress for {idle:.0f} s in phase '
                      f'"{_PHASE[0]}"; exiting (124)', file=sys.stderr, flush=True)
                os._exit(124)
    threading.Thread(target=run, daemon=True).start()


def synth_table(n, seed, device):
    """SURVEY.md 8d distributions: 95% positions ~N(0,10^2), 5% in a 1e-3 cube
    (forces equal-key Morton runs > 256); f_dc ~N(0,1); f_rest ~N(0,0.1^2);
    opacity ~N(0,2^2); scale ~U(-7,-2); rot ~N(0,1)^4 (not normalised)."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    f = dict(device=device, dtype=torch.float32)
    cols = {}
    cube = torch.rand(n, generator=g, **f) < 0.05
    for a, off in zip('xyz', (1.0, -2.0, 3.0)):
        v = torch.randn(n, generator=g, **f) * 10
        c = off + torch.rand(n, generator=g, **f) * 1e-3
        cols[a] = torch.where(cube, c, v).contiguous()
    for i in range(3):
        cols[f'f_dc_{i}'] = torch.randn(n, generator=g, **f)
    for i in range(45):
        cols[f'f_rest_{i}'] = torch.randn(n, generator=g, **f) * 0.1
    cols['opacity'] = torch.randn(n, generator=g, **f) * 2
    for i in range(3):
        cols[f'scale_{i}'] = torch.rand(n, generator=g, **f) * 5 - 7
    for i in range(4):
        cols[f'rot_{i}'] = torch.randn(n, generator=g, **f)
    return cols


def cpu_baseline(args):
    """Time the CPU restatement (oracle/, the reference algorithm in C) on a bounded sample and
    extrapolate to the bench workload: 1 thread (the reference is single-threaded JS) and every
    host core this job may use (OpenMP over points: assign and the SH0 pipeline's 1-D k-means)."""
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    import numpy as np

    import oracle
    oracle.build()
    rng = np.random.default_rng(1002)
    K, D = 65536, 45
    # (a) one clusterKdTreeCpu pass at K = 65,536 over a fixed point sample; centroids are data
    # rows (the reference's init, k-means.ts:8-20)
    n1, nmt = args.cpu_assign_sample, args.cpu_assign_sample_mt
    data = [rng.normal(0, 0.1, K + max(n1, nmt)).astype(np.float32) for _ in range(D)]
    cen = np.stack([c[:K] for c in data])
    oracle.set_threads(1)
    t0 = time.perf_counter()
    rc, lab1 = oracle.kmeans_assign([c[K:K + n1] for c in data], cen)
    ta = (time.perf_counter() - t0) / n1
    # the same assign on every host core this job may use; the box sets OMP_NUM_THREADS to its CPU
    # share.  The first n1 labels must equal the 1-thread ones.
    threads = int(os.environ.get('OMP_NUM_THREADS') or os.cpu_count() or 1)
    t0 = time.perf_counter()
    rc_mt, lab_mt = oracle.kmeans_assign([c[K:K + nmt] for c in data], cen, threads=threads)
    ta_mt = (time.perf_counter() - t0) / nmt
    same = bool(np.array_equal(np.asarray(lab_mt)[:min(n1, nmt)], np.asarray(lab1)[:min(n1, nmt)]))
    # (b) everything else: the SH0 writeSog pipeline (Morton, means/quats, two cluster1d k-means of
    # 10 iterations, textures) on a splat sample, 1 thread and then with the assign loops threaded
    n = args.cpu_rest_sample
    names = ['x', 'y', 'z', 'f_dc_0', 'f_dc_1', 'f_dc_2', 'opacity', 'scale_0', 'scale_1', 'scale_2',
             'rot_0', 'rot_1', 'rot_2', 'rot_3']
    cols = {k: rng.normal(0, 1, n).astype(np.float32) for k in names}
    t0 = time.perf_counter()
    oracle.sog(cols, 0, args.iters, oracle.mulberry32(3, 200_000))
    tb = (time.perf_counter() - t0) / n
    oracle.set_threads(threads)
    try:
        t0 = time.perf_counter()
        oracle.sog(cols, 0, args.iters, oracle.mulberry32(3, 200_000))
        tb_mt = (time.perf_counter() - t0) / n
    finally:
        oracle.set_threads(1)
    per_splat = args.iters * ta + tb
    per_splat_mt = args.iters * ta_mt + tb_mt
    all_cores = {
        'value': 1e-6 / per_splat_mt,
        'unit': 'Msplats/s',
        'cores': threads,
        'kind': 'port',
        'sample': (f'oracle/ C restatement on {threads} OpenMP threads: KdTree assign at K=65536, D=45 on a fixed '
                   f'{nmt}-point sample ({ta_mt * 1e3:.3f} ms/point/iter, labels of the first {min(n1, nmt)} equal '
                   f'to the 1-thread run: {same}) x {args.iters} iters + SH0 writeSog pipeline with threaded assign '
                   f'loops on {n} splats ({tb_mt * 1e6:.2f} us/splat); extrapolated per splat'),
    }
    return {
        'value': 1e-6 / per_splat,
        'unit': 'Msplats/s',
        'cores': 1,
        'kind': 'port',
        'sample': (f'oracle/ C restatement, 1 thread: KdTree assign at K=65536, D=45 timed on a fixed {n1}-point '
                   f'sample ({ta * 1e3:.2f} ms/point/iter) x {args.iters} iters + SH0 writeSog pipeline timed on '
                   f'{n} splats ({tb * 1e6:.2f} us/splat); extrapolated per splat'),
    }, all_cores


def realistic_table(n, seed, device, zero_frac=0.3, clumps=20_000, clump_frac=0.8):
    """north_star's table shape with the distributions trained scenes bring:
    SH rows heavy-tailed and correlated -- Student-t (nu = 3) through a fixed mixing matrix, the
    t3 rows of tests/test_gpu_parity.py -- with `zero_frac` of them all zero (splats whose SH
    never trained: exact duplicates), and `clump_frac` of the positions in `clumps` tight clumps
    (Morton recursion, equal keys).  The other columns as synth_table."""
    import torch
    cols = synth_table(n, seed, device)
    g = torch.Generator(device=device)
    g.manual_seed(seed + 7)
    f = dict(device=device, dtype=torch.float32)
    cid = torch.randint(0, clumps, (n,), generator=g, device=device)
    inclump = torch.rand(n, generator=g, **f) < clump_frac
    for a in 'xyz':
        centre = torch.randn(clumps, generator=g, **f) * 10
        cols[a] = torch.where(inclump, centre[cid] + torch.randn(n, generator=g, **f) * 1e-3, cols[a]).contiguous()
    D = 45
    m = torch.eye(D, device=device) + 0.5 * torch.randn(D, D, generator=g, **f) / D ** 0.5
    zero = torch.rand(n, generator=g, **f) < zero_frac
    for a in range(0, n, 1 << 21):
        b = min(n, a + (1 << 21))
        t = torch.randn(b - a, D, generator=g, **f)
        chi = (torch.randn(b - a, 3, generator=g, **f) ** 2).sum(1, keepdim=True) / 3
        sh = (t / chi.sqrt()) @ m.T * 0.1
        sh[zero[a:b]] = 0
        for i in range(D):
            cols[f'f_rest_{i}'][a:b] = sh[:, i]
    return cols


PLY_ORDER = (['x', 'y', 'z', 'nx', 'ny', 'nz', 'f_dc_0', 'f_dc_1', 'f_dc_2'] + [f'f_rest_{i}' for i in range(45)] +
             ['opacity', 'scale_0', 'scale_1', 'scale_2', 'rot_0', 'rot_1', 'rot_2', 'rot_3'])


def end_to_end(ctx, cols, iters, draws, tex, ref_archive, meta, reps=3):
    """The CLI's work for `splat-transform in.ply out.sog` on this table: the step's table is
    written once as a binary little-endian 3DGS PLY (62 float properties, 248 B per splat,
    normals 0; untimed), then each timed rep reads the file into device columns
    (st_dev_ply_read: page cache -> pinned chunks -> HBM -> k_ply_cols), runs the same
    writeSog step, builds the .sog archive (WebP x7 + CRC + ZIP) and writes it to a file.
    The archive must equal the in-memory step's byte for byte."""
    import tempfile

    import numpy as np
    import torch
    n = cols['x'].shape[0]
    d = tempfile.mkdtemp(prefix='st_e2e_', dir=os.environ.get('TMPDIR', '/tmp'))
    src, dst = os.path.join(d, 'in.ply'), os.path.join(d, 'out.sog')
    try:
        head = ('ply\nformat binary_little_endian 1.0\n' + f'element vertex {n}\n' +
                ''.join(f'property float {k}\n' for k in PLY_ORDER) + 'end_header\n').encode()
        zero = torch.zeros(n, dtype=torch.float32, device=cols['x'].device)
        with open(src, 'wb') as f:
            f.write(head)
            step = 1 << 22
            for a in range(0, n, step):
                b = min(n, a + step)
                rows = torch.stack([(cols[k][a:b] if k in cols else zero[a:b]) for k in PLY_ORDER], 1)
                f.write(rows.cpu().numpy().tobytes())
        del zero
        file_bytes = os.path.getsize(src)

        def run(streamed):
            times, parts, same = [], [], True
            for r in range(reps + 1):  # rep 0 warms the file cache and the ingest buffers
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                _, els = ctx.read_ply_dev(src)
                vc = dict(els)['vertex']
                table = {k: v for k, v in vc.items() if not k.startswith('n')}
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                if streamed:  # st_dev_sog_file: the archive streamed to the file beside the SH k-means
                    _, _, size = ctx.dev_sog_file(table, iters, draws, tex, dst)
                    t2 = t3 = t4 = time.perf_counter()
                else:
                    meta, _ = ctx.dev_sog(table, iters, draws, tex)
                    t2 = time.perf_counter()
                    addr, size = ctx.dev_sog_bundle_view(meta, n, tex, 0, 0)
                    t3 = time.perf_counter()
                    fd = os.open(dst, os.O_WRONLY | os.O_CREAT, 0o644)  # as dev_sog_file: no O_TRUNC
                    try:
                        mv, o = memoryview((ctypes_char_array(size)).from_address(addr)).cast('B'), 0
                        while o < size:
                            o += os.write(fd, mv[o:])
                        os.ftruncate(fd, size)
                    finally:
                        os.close(fd)
                    t4 = time.perf_counter()
                if r:
                    times.append(t4 - t0)
                    parts.append((t1 - t0, t2 - t1, t3 - t2, t4 - t3))
                del els, vc, table
                same = same and (open(dst, 'rb').read() == ref_archive)
            i = sorted(range(len(times)), key=lambda j: times[j])[len(times) // 2]
            ms = times[i] * 1e3
            split = (dict(ply_ingest=parts[i][0] * 1e3, sog_step_archive_file=parts[i][1] * 1e3) if streamed else
                     dict(zip(('ply_ingest', 'sog_step', 'container', 'file_write'), (x * 1e3 for x in parts[i]))))
            return {'ms': ms, 'Msplats_per_s': n / ms / 1e3, 'split_ms': split, 'sog_bytes': size,
                    'archive_equals_in_memory_step': same}

        one = run(True)
        sep = run(False)
        return {'what': 'PLY file (page cache) -> device columns -> writeSog step -> .sog archive -> file, rank 0 '
                        '(st_dev_sog_file: the five textures final before the SH k-means are encoded and written '
                        'while it runs)',
                'ply_bytes': file_bytes, 'sog_bytes': one['sog_bytes'], 'ms': one['ms'],
                'Msplats_per_s': one['Msplats_per_s'], 'split_ms': one['split_ms'], 'reps': reps,
                'archive_equals_in_memory_step': one['archive_equals_in_memory_step'] and
                sep['archive_equals_in_memory_step'],
                'separate_calls': dict(sep, what='st_dev_sog, st_dev_sog_bundle_view, one write(2)'),
                'node_host': node_end_to_end(ctx, src, dst, n, iters, reps, draws, tex, meta)}
    finally:
        for f in (src, dst):
            if os.path.exists(f):
                os.remove(f)
        os.rmdir(d)


NODE_CLOCK = [2024, 0, 1, 0, 0, 0]  # the Node job's pinned Date: 2024-01-01 00:00:00
NODE_DOS_TIME, NODE_DOS_DATE = 0, ((2024 - 1980) << 9) | (1 << 5) | 1  # zip-writer.ts:39-41 of that clock


def node_end_to_end(ctx, src, dst, n, iters, reps, draws, tex, meta):
    """The same job through the Node drop-in host (tools/bench_node.js: js/index.js readPly ->
    writeSogFile over the N-API addon, as the reference's index.ts:433-510 drives its reader and
    writer): the PLY read into a host DataTable, then uploaded and written as .sog.  A separate
    process on the same GPU; None when node or the addon is absent.  Math.random is the bench's
    draw stream and Date a pinned clock in every rep, so each timed rep's file must equal the
    library's archive of the main step's textures with that clock (archive_equals_library)."""
    import hashlib
    import shutil
    import subprocess

    import numpy as np
    node = shutil.which('node')
    addon = os.path.join(ROOT, 'splat-transform_amd', 'napi', 'build', 'addon.node')
    if not node or not os.path.exists(addon):
        return None
    dfile = dst + '.draws.f64'
    np.asarray(draws, '<f8').tofile(dfile)
    try:
        r = subprocess.run([node, '--expose-gc', os.path.join(ROOT, 'tools', 'bench_node.js'), src, dst, str(max(3, reps)),
                            str(iters),
                            dfile, json.dumps(NODE_CLOCK)], capture_output=True, text=True, timeout=600)
    finally:
        os.remove(dfile)
    if r.returncode != 0:
        return {'error': r.stderr[-2000:]}
    out = json.loads(r.stdout.strip().splitlines()[-1])
    want = None
    if meta is not None:
        addr, size = ctx.dev_sog_bundle_view(meta, n, tex, NODE_DOS_TIME, NODE_DOS_DATE)
        want = hashlib.sha256(bytes((ctypes_char_array(size)).from_address(addr))).hexdigest()
    runs = sorted(out['runs'], key=lambda x: x['total'])
    med = runs[len(runs) // 2]
    return {'what': 'node tools/bench_node.js: readPly(FileHandle) -> host DataTable -> writeSogFile(FileHandle) '
                    '(js/index.js over napi/addon.node: st_ply_read_resident + st_sog_file; the columns JS never reads stay '
                    'in HBM), median of the timed reps; '
                    'Math.random = the bench\'s draw stream, Date pinned; global.gc() between reps (untimed), so '
                    'every rep\'s columns reuse the addon\'s faulted-in blocks',
            'ms': med['total'], 'Msplats_per_s': n / med['total'] / 1e3,
            'split_ms': {'readPly': med['readPly'], 'writeSogFile': med['writeSogFile']},
            'rows': out['rows'], 'sog_bytes': out['sog_bytes'], 'reps': len(runs),
            'resident_columns_reused': med.get('reusedColumns'),
            'archive_sha256': out['sha256'][-1],
            'archive_equals_library': (want is not None and all(h == want for h in out['sha256'])),
            'how_checked': 'sha256 of the file after every rep (warm-up included) against st_dev_sog_bundle_view of '
                           'the main step\'s textures and meta with the same DOS clock'}


def check_labels(sh, prev, lab, n_labels, g):
    """sampled points: is the label the exact f64 argmin over `prev` (kd-tree.ts:26-33 order)?
    returns (wrong labels, exact ties -- the KdTree order decides those, not checked)"""
    import torch
    dev = sh.device
    d, k = prev.shape
    n = lab.shape[0]
    if n == 0:
        return 0, 0
    pts = torch.randint(0, n, (n_labels,), generator=g).to(dev)
    lab64 = lab.long()
    pd_all = sh[:, pts].double()
    cd = prev.double()
    bad, ties = 0, 0
    for s in range(0, n_labels, 256):
        e = min(n_labels, s + 256)
        dist = torch.zeros(e - s, k, dtype=torch.float64, device=dev)
        for j in range(d):
            v = cd[j][None, :] - pd_all[j, s:e][:, None]
            dist += v * v
        mn = dist.min(1).values
        got = dist.gather(1, lab64[pts[s:e], None]).squeeze(1)
        bad += int((got != mn).sum().item())
        ties += int(((dist == mn[:, None]).sum(1) > 1).sum().item())
    return bad, ties


def check_all_labels(sh, prev, lab, tile=8192):
    """every point: is its label the exact f64 argmin over `prev` (kd-tree.ts:26-33)?  Scores
    |c|^2 - 2 p.c from an f64 GEMM (torch, independent of the library's kernels) decide every
    point whose two best scores are apart by more than twice a bound on the GEMM's error; the
    others take the reference's own distance (sequential f64 sum of (c - p)^2 over the dims)
    against every centroid within that window.  Returns (wrong labels, exact ties unchecked,
    points decided by the sequential distances)."""
    import torch
    d, k = prev.shape
    n = lab.shape[0]
    cd = prev.double()
    cn = (cd * cd).sum(0)
    cmax = float(cn.max().sqrt())
    # each score's GEMM error is <= ~(d + 2) u (|c|^2 + 2 |p| |c|) and the reference's sequential
    # f64 distance is within ~(d + 2) u |p - c|^2 <= (d + 2) u (|p| + |c|)^2 of the exact one
    # (u = 2^-53): scores apart by more than twice 64 x (d + 2) u 2 (|p| + max|c|)^2 keep their order
    rel = 64 * (d + 2) * 2.0 ** -53
    bad = ties = slow = 0
    lab64 = lab.long()
    for s in range(0, n, tile):
        e = min(n, s + tile)
        p = sh[:, s:e].double()
        pn = (p * p).sum(0).sqrt()
        score = torch.addmm(cn[None, :], p.t(), cd, beta=1.0, alpha=-2.0)
        m1, i1 = score.min(1)
        rows = torch.arange(e - s, device=sh.device)
        best = score[rows, i1].clone()
        score[rows, i1] = float('inf')
        m2 = score.min(1).values
        score[rows, i1] = best
        w = rel * 2 * (pn + cmax) ** 2
        clear = (m2 - m1) > 2 * w
        bad += int(((lab64[s:e] != i1) & clear).sum().item())
        amb = torch.nonzero(~clear).squeeze(1)
        slow += amb.numel()
        for a0 in range(0, amb.numel(), 1024):  # the reference's own distances over the windows' rows
            a = amb[a0:a0 + 1024]
            row, col = torch.nonzero(score[a] <= (m1[a] + 2 * w[a])[:, None], as_tuple=True)
            dist = torch.zeros(row.numel(), dtype=torch.float64, device=sh.device)
            for j in range(d):  # dimension by dimension, as kd-tree.ts:26-33 sums
                v = cd[j, col] - p[j, a[row]]
                dist = dist + v * v
            mn = torch.full((a.numel(),), float('inf'), dtype=torch.float64, device=sh.device)
            mn = mn.scatter_reduce(0, row, dist, reduce='amin')
            at_min = dist == mn[row]
            nmin = torch.zeros(a.numel(), dtype=torch.long, device=sh.device).scatter_add(0, row, at_min.long())
            # the unique minimum's column per row (rows with a tie are counted, not checked)
            win = torch.full((a.numel(),), -1, dtype=torch.long, device=sh.device)
            win = win.scatter_reduce(0, row[at_min], col[at_min], reduce='amax')
            ties += int((nmin > 1).sum().item())
            bad += int(((nmin == 1) & (win != lab64[s + a])).sum().item())
        del score
    return bad, ties, slow


def verify_sharded(ctx, local_sh, tex, step, n_labels=2048, seed=7, all_labels=False):
    """the sharded step's output (every rank): the library's k-means snapshot on a re-run; this
    rank's labels (sampled, or all with all_labels) are exact f64 argmins over the last assign's
    centroids, every rank holds the same final centroids, and rank 0's textures equal the last
    timed step's"""
    import torch
    import torch.distributed as dist
    before = {k: v.clone() for k, v in tex.items()} if tex else None
    ctx.set_verify(True)
    try:
        step()
        torch.cuda.synchronize()
    finally:
        ctx.set_verify(False)
    same = all(torch.equal(before[k], tex[k]) for k in tex) if tex else True
    prev, cen, lab = ctx.verify_snapshot(local_sh.device)
    g = torch.Generator(device='cpu')
    g.manual_seed(seed + dist.get_rank())
    if all_labels:
        bad, ties, _ = check_all_labels(local_sh, prev, lab)
        n_labels = lab.shape[0]
    else:
        bad, ties = check_labels(local_sh, prev, lab, n_labels, g)
    ref = cen.clone()
    dist.broadcast(ref, 0)
    same_cen = bool(torch.equal(ref, cen))
    t = torch.tensor([bad, ties, 0 if same else 1, 0 if same_cen else 1, n_labels], dtype=torch.float64,
                     device=local_sh.device)
    dist.all_reduce(t)
    same_cen = int(t[3].item()) == 0
    ok = int(t[0].item()) == 0 and int(t[2].item()) == 0 and same_cen
    return {'ok': ok, 'labels_checked': int(t[4].item()), 'labels_wrong': int(t[0].item()),
            'label_exact_ties_unchecked': int(t[1].item()), 'textures_equal_timed_step': int(t[2].item()) == 0,
            'centroids_identical_on_every_rank': same_cen,
            'how': 'snapshot of the sharded SH palette k-means (st_ctx_set_verify) on a re-run of the step; '
                   'each rank checks its labels as exact f64 argmins over the last assign\'s centroids'}


def verify_step(ctx, cols, tex, step, n_labels=4096, n_clusters=64, seed=7, all_labels=False):
    """Re-run the step with the library's k-means snapshot on (outside the timed region) and
    check its output against the reference's definitions (k-means.ts:137-201, kd-tree.ts:22-70):
      * the textures equal those of the last timed step (the verified step IS the timed one);
      * sampled SH labels are exact f64 argmins (sequential sum of (c - p)^2 over the 45 dims,
        kd-tree.ts:26-33) over the centroids the last assign used; an exact tie (KdTree order
        decides) is counted, not checked;
      * sampled centroids are the f32-rounded sequential f64 means of their members in
        ascending point order (calcAverage, k-means.ts:41-63);
      * every shN_labels texel holds the label of the row at its Morton position.
    all_labels: every label instead of a sample (check_all_labels, a few seconds at 10M)."""
    import numpy as np
    import torch
    dev = cols['x'].device
    before = {k: v.clone() for k, v in tex.items()}
    ctx.set_verify(True)
    try:
        step()
        torch.cuda.synchronize()
    finally:
        ctx.set_verify(False)
    same = all(torch.equal(before[k], tex[k]) for k in tex)
    del before
    prev, cen, lab = ctx.verify_snapshot(dev)
    d, k = prev.shape
    n = lab.shape[0]
    sh = torch.stack([cols[f'f_rest_{i}'] for i in range(d)])  # [d, n] f32
    g = torch.Generator(device='cpu')
    g.manual_seed(seed)
    slow = None
    if all_labels:
        bad_labels, ties, slow = check_all_labels(sh, prev, lab)
        n_labels = n
    else:
        bad_labels, ties = check_labels(sh, prev, lab, n_labels, g)
    lab64 = lab.long()
    # centroids: sequential f64 mean of the members (numpy cumsum is a left-to-right chain)
    counts = torch.bincount(lab64, minlength=k)
    nonempty = torch.nonzero(counts > 0).squeeze(1)
    pick = nonempty[torch.randperm(nonempty.numel(), generator=g)[:n_clusters - 1].to(dev)]
    pick = torch.cat([pick, torch.argmax(counts)[None]])
    bad_cen = 0
    cen_h = cen.cpu().numpy()
    for c in pick.tolist():
        members = torch.nonzero(lab64 == c).squeeze(1)
        vals = sh[:, members].double().cpu().numpy()
        mean = (np.cumsum(vals, axis=1)[:, -1] / members.numel()).astype(np.float32)
        bad_cen += int((mean.view(np.uint32) != cen_h[:, c].view(np.uint32)).sum())
    # texels: shN_labels[i] = label of the row at Morton position i (write-sog.ts:338-348)
    order = torch.arange(n, dtype=torch.int32, device=dev)  # generateIndices (write-sog.ts:42-49)
    ctx.dev_morton_order(cols['x'], cols['y'], cols['z'], order)
    ctx.synchronize()
    t = tex['shN_labels'].view(-1, 4)[:n].long()
    tl = t[:, 0] | (t[:, 1] << 8)
    bad_texels = int((tl != (lab64[order.long()] & 0xffff)).sum().item())
    ok = same and bad_labels == 0 and bad_cen == 0 and bad_texels == 0
    out = {'ok': ok, 'textures_equal_timed_step': same, 'labels_checked': n_labels, 'labels_wrong': bad_labels,
           'label_exact_ties_unchecked': ties, 'clusters_checked': len(pick), 'centroid_values_wrong': bad_cen,
           'empty_clusters': int((counts == 0).sum().item()), 'texel_labels_checked': n,
           'texel_labels_wrong': bad_texels,
           'how': 'snapshot of the SH palette k-means (st_ctx_set_verify) on a re-run of the step; f64 argmin '
                  'over the last assign\'s centroids, sequential f64 member means, Morton texel placement'}
    if slow is not None:
        out['labels_decided_by_sequential_distance'] = slow
    return out


def ctypes_char_array(size):
    import ctypes
    return ctypes.c_char * size


def sog_stage_table(stages, n, iters, K=65536, D=45):
    """writeSog's top-level stages (the stage-marked step) priced by their algorithmic work
    (SURVEY 8d): HBM bytes per splat for the memory-bound ones, dot-product flops for the SH
    palette k-means (whose sweep is MFMA-bound; its HBM bytes are listed too)"""
    if not stages:
        return None
    cb = K * D  # values of the codebook cluster1d (the palette's centroid coordinates)
    spec = {
        'sog.cluster1d': ('hbm', 30 * iters * n + 4 * n,
                          'the scales and the colours cluster1d side by side (st_sog.hip): 5 B per '
                          'value-iteration (4 B read + 1 B label) x 6 values + the opacity read'),
        'sog.shkmeans': ('mfma', 2.0 * n * K * D * iters, 'SH palette k-means: 2 n K D flop per iteration '
                         '(the sweep); 184 B/splat/iter of HBM besides; the Morton order (92 B/splat) and '
                         'the five textures (40 + 14 B/splat) run beside it on a side context'),
        'sog.shn': ('hbm', 5 * iters * cb + 8 * n, 'codebook cluster1d over K x D values + shN labels texels'),
    }
    out = {}
    for k, (bound, work, what) in spec.items():
        ms = stages.get(k)
        if ms is None or ms <= 0:
            continue
        if bound == 'hbm':
            gbs = work / (ms / 1e3) / 1e9
            out[k] = {'ms': ms, 'bound': 'hbm', 'alg_bytes': work, 'achieved_GBps': gbs,
                      'frac_hbm': gbs / (HBM_TBPS * 1e3), 'work': what}
        else:
            tf = work / (ms / 1e3) / 1e12
            out[k] = {'ms': ms, 'bound': 'mfma', 'alg_flops': work, 'achieved_TFLOPs': tf,
                      'frac_peak': tf / MFMA_F16_DENSE_TFLOPS, 'work': what}
    return out


BLOCK = 10_000_000  # rows per fixed-seed block of the synthetic tables
SEED = 1002


def table_rows(T, lo, hi, dev, seed=SEED, block=BLOCK):
    """rows [lo, hi) of the T-row synthetic table whose block b (rows [b*block, (b+1)*block)) is
    synth_table(rows in the block, seed + b): the same T-row table whatever the rank split"""
    import torch
    parts = []
    for b in range(lo // block, (hi - 1) // block + 1) if hi > lo else ():
        a, e = b * block, min(T, (b + 1) * block)
        full = synth_table(e - a, seed + b, dev)
        if lo <= a and e <= hi:
            parts.append(full)
        else:
            parts.append({k: v[max(lo, a) - a:min(hi, e) - a].clone() for k, v in full.items()})
        del full
    if not parts:
        return synth_table(0, seed, dev)
    if len(parts) == 1:
        return parts[0]
    out = {k: torch.cat([p[k] for p in parts]) for k in parts[0]}
    del parts
    return out


NORTH_STAR_SPLATS = 10_000_000  # BASELINE.json north_star: "a synthetic 10M-splat input at 1 GPU and its 2/4/8-GPU
CONFIG4_SPLATS = 50_000_000     # scaling curve"; BASELINE config 4: one 50M-splat table


def workload(args, world):
    """(description, splats in the job, scaling) of the run's main record: a function of the flags
    only, so the same workload prints the same `config.workload` at every N (the split goes into
    `config.parallelism`)"""
    it = f'{args.iters} k-means iters'
    if args.merge:
        F, S = args.merge, args.file_splats
        return (f'config 5: merge {F} x {S / 1e6:g}M-splat inputs (combine, seeds 5001..) + Morton -> writeSog SH3, '
                f'{it}'), F * S, 'strong'
    if args.splats is not None:
        return f'writeSog SH3, {args.splats} splats per GPU (fixed-seed 10M blocks), {it}', args.splats * world, 'weak'
    T = args.total_splats if args.total_splats is not None else NORTH_STAR_SPLATS
    what = ('north_star: ' if T == NORTH_STAR_SPLATS else 'config 4: ' if T == CONFIG4_SPLATS else '')
    return f'{what}writeSog SH3 of one {T / 1e6:g}M-splat table (fixed-seed 10M blocks, seed 1002), {it}', T, 'strong'


def rank_tables(args, world, rank, dev):
    """this rank's input tables (device columns) and the workload's description"""
    desc, total, scaling = workload(args, world)
    if args.merge:
        F, S = args.merge, args.file_splats
        lo, hi = total * rank // world, total * (rank + 1) // world
        tabs = []
        for f in range(F):
            a, b = max(lo, f * S), min(hi, (f + 1) * S)
            if b > a or (f == F - 1 and not tabs):
                full = synth_table(S, 5001 + f, dev)  # merge inputs use seeds 5001..
                tabs.append({k: v[a - f * S:max(a, b) - f * S].contiguous() for k, v in full.items()})
                del full
        return tabs, total, desc, scaling
    if scaling == 'weak':
        n = args.splats
        return [table_rows(total, n * rank, n * (rank + 1), dev)], total, desc, scaling
    lo, hi = total * rank // world, total * (rank + 1) // world
    return [table_rows(total, lo, hi, dev)], total, desc, scaling


TEX_ORDER = ('means_l', 'means_u', 'quats', 'scales', 'sh0', 'shN_labels', 'shN_centroids')


def textures_digest(tex, meta):
    """sha256 over the seven textures (write-sog.ts order) and the meta fields: equal for every N"""
    import hashlib

    import numpy as np
    h = hashlib.sha256()
    for k in TEX_ORDER:
        if k in tex:
            h.update(tex[k].cpu().numpy().tobytes())
    if meta is not None:
        for f in ('width', 'height', 'sh_bands', 'palette_size', 'shn_width', 'shn_height'):
            h.update(int(getattr(meta, f)).to_bytes(8, 'little'))
        for f in ('means_min', 'means_max', 'scales_codebook', 'sh0_codebook', 'shn_codebook'):
            h.update(np.array(list(getattr(meta, f)), np.float64).tobytes())
    return h.hexdigest()


_PHASE = ['start']


def heartbeat(period=30.0):
    """a progress line on stderr every `period` s: the long quiet phases (the CPU baseline's ~2 min
    of single-thread KdTree work, the table builds) never look like a hung run"""
    import threading
    t0 = time.time()

    def run():
        while True:
            time.sleep(period)
            print(f'bench.py: {_PHASE[0]} ({time.time() - t0:.0f} s)', file=sys.stderr, flush=True)
    threading.Thread(target=run, daemon=True).start()


def torch_backend(args):
    """the torch.distributed backend of a sharded run: the library carries every collective of the step
    (its own RCCL communicators, or host shared memory under --backend gloo), so torch's process
    group only serves bench.py between steps and runs on gloo -- torch's bundled RCCL is then
    loaded but never initialised, and each rank runs one RCCL (st_rccl.cpp's).  --dist-python's
    step is torch.distributed collectives: --backend there."""
    if args.torch_backend != 'auto':
        return args.torch_backend
    return args.backend if args.dist_python else 'gloo'


def main(args):
    import numpy as np
    import torch
    import torch.distributed as dist

    import splat_hip as sh

    heartbeat()
    progress('started')

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    local = local % max(torch.cuda.device_count(), 1)  # ranks > GPUs only in a gloo rehearsal
    if world > 1 and args.backend == 'nccl' and torch.cuda.device_count() < world:
        raise SystemExit(f'bench.py: {world} RCCL ranks need {world} GPUs, this node has {torch.cuda.device_count()} '
                         '(rehearse several ranks on one GPU with --backend gloo: the library\'s host shared-memory '
                         'transport)')
    if world > 1:
        rank_watchdog(args.rank_watchdog)
    torch.cuda.set_device(local)  # before the process group: RCCL binds the rank to this device
    # N = 1 runs st_dev_sog unless asked for the sharded path (--dist / --dist-python) or given several
    # input tables (--merge: combine inside st_dev_sog_sharded)
    sharded = world > 1 or args.dist or args.dist_python or bool(args.merge)
    if sharded:
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        os.environ.setdefault('MASTER_PORT', '29533')
        dist.init_process_group(torch_backend(args), init_method='env://', rank=rank, world_size=world)
    dev = torch.device('cuda', local)

    # one real stream for the library and the torch glue (st_ctx_set_stream(NULL) would select the
    # context's own stream, and torch's legacy default stream has handle 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx = sh.Context(local)
    ctx.set_stream(stream.cuda_stream)
    # the host's Math.random stream (any uniform [0,1) doubles; the reference uses Math.random):
    # one stream for the whole job, identical on every rank
    draws = np.random.default_rng(42).random(2 * 65536 * (args.iters + 2))
    comm = None
    if sharded and not args.dist_python:
        if args.backend == 'gloo':
            # several ranks on one GPU: the library's host shared-memory transport (st_comm_init_host),
            # the same st_dev_sog_sharded calls; torch.distributed hands out the job's name
            import uuid
            name = [f'bench-{uuid.uuid4().hex[:16]}' if rank == 0 else None]
            dist.broadcast_object_list(name, src=0)
            comm = sh.Comm.host(ctx, world, rank, name[0])
        else:
            # the library's own RCCL communicator (st_comm_init_rank); torch.distributed hands out the id
            uid = [sh.comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            comm = sh.Comm(ctx, world, rank, uid[0])

    def make_step(tabs, total):
        """the step closure over this rank's tables and rank 0's device outputs"""
        W, H, pal, cw, ch = sh.sog_geometry(total, 15)
        tex = None
        if rank == 0:
            u8 = dict(device=dev, dtype=torch.uint8)
            tex = {k: torch.empty(W * H * 4, **u8) for k in ('means_l', 'means_u', 'quats', 'scales', 'sh0',
                                                            'shN_labels')}
            tex['shN_centroids'] = torch.empty(cw * ch * 4, **u8)
        last = {}
        if not sharded:
            def step():
                return ctx.dev_sog(tabs[0], args.iters, draws, tex)
        elif not args.dist_python:
            def step():
                return ctx.dev_sog_sharded(comm, tabs, args.iters, draws, tex)
        else:
            import splat_dist
            ops = splat_dist.HipOps(ctx, dev)
            pcomm = splat_dist.Comm()
            cols = tabs[0] if len(tabs) == 1 else {k: torch.cat([t[k] for t in tabs]) for k in tabs[0]}

            def step():
                t_, m_, used = splat_dist.write_sog(ops, pcomm, cols, args.iters, draws)
                last.update(tex=t_, meta=m_)
                if rank == 0:
                    for k in tex:
                        tex[k].copy_(t_[k])
                return (splat_dist.meta_struct(m_) if rank == 0 else None), used
        return step, tex, pal

    def timed(step, steps, warmup):
        for i in range(warmup):
            step()
            progress(f'warmup step {i + 1}/{warmup}')
        if sharded:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            meta, used = step()
            progress(f'timed step {i + 1}/{steps}')
        torch.cuda.synchronize()
        if sharded:
            dist.barrier()
        el = time.perf_counter() - t0
        if sharded:
            t = torch.tensor([el], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = t.item()
        return el, meta, used

    if comm:
        rccl_ranks = comm.count() if comm.transport == 'rccl' else None
        transport = comm.transport
    else:
        rccl_ranks = world if sharded and args.backend == 'nccl' else None
        transport = ('torch.distributed ' + torch_backend(args)) if sharded else None
    devices = None
    if sharded:
        devs = [None] * world
        dist.all_gather_object(devs, (os.uname().nodename, local))
        devices = len(set(str(d) for d in devs))
    progress('building the tables')
    tabs, total, wl_desc, scaling = rank_tables(args, world, rank, dev)
    step, tex, pal = make_step(tabs, total)
    torch.cuda.synchronize()
    progress('warmup steps')
    for i in range(args.warmup):
        step()
        progress(f'warmup step {i + 1}/{args.warmup}')
    progress('timed steps')
    ctx.set_profiling(True)
    ctx.reset_kernel_stats()
    os.environ.pop('ST_TIMING', None)
    elapsed, meta, used = timed(step, args.steps, 0)
    # the last timed step's SH palette k-means: how its points were decided (summed over its 10
    # assigns; the python harness path runs its own k-means and leaves this empty)
    sh_assign = ctx.kmeans_stats() or None
    sweep_ms, sweep_launches = ctx.kernel_stats('kn.sweep')
    kstats = {}
    for name in ('kn.sweep', 'kn.collect', 'kn.fixrow', 'kn.fixpair', 'kn.exact', 'kn.sumnd', 'k1.assign', 'k1.sum',
                 'chunk.pack'):
        ms, cnt = ctx.kernel_stats(name)
        kstats[name] = {'avg_ms': ms / max(cnt, 1), 'launches': cnt}
    ctx.set_profiling(False)
    n_local = sum(t['x'].shape[0] for t in tabs)

    # one more step with per-stage event marks (outside the timed region; single device only)
    stages = None
    if not sharded:
        os.environ['ST_TIMING'] = '1'
        step()
        torch.cuda.synchronize()
        stages = json.loads(ctx.timings())
        os.environ.pop('ST_TIMING', None)

    # the last timed step's output checked against the reference's definitions
    verification = None
    progress('stage table and verification')
    if not args.no_verify:
        if not sharded:
            verification = verify_step(ctx, tabs[0], tex, step, all_labels=not args.verify_sample)
        elif not args.dist_python:
            local_sh = torch.stack([torch.cat([t[f'f_rest_{i}'] for t in tabs]) for i in range(45)])
            verification = verify_sharded(ctx, local_sh, tex, step, all_labels=not args.verify_sample)
            del local_sh

    # extra records beside the main one (fewer steps; outside the main timed region)
    extras = {}
    main_default = not args.merge and args.splats is None and args.total_splats is None and not args.dist_python
    if main_default and not args.no_extra:
        ks, kw = max(1, args.extra_steps), 1
        main_sha = textures_digest(tex, meta) if rank == 0 else None

        def record(what, T, el, scal, sha=None):
            r = {'workload': what, 'splats_total': T, 'value': T * ks / el / 1e6, 'unit': 'Msplats/s',
                 'ms_per_step': el / ks * 1e3, 'steps': ks, 'warmup': kw, 'scaling': scal}
            if sha is not None:
                r['textures_sha256'] = sha
            return r
        if not sharded:
            # the same table through the sharded code path at world 1 (one-rank RCCL communicator): the
            # denominator of a scaling curve taken over st_dev_sog_sharded alone
            progress('extra record: sharded path at world 1')
            comm1 = sh.Comm(ctx, 1, 0, sh.comm_unique_id())
            W1, H1, _, cw1, ch1 = sh.sog_geometry(total, 15)
            u8 = dict(device=dev, dtype=torch.uint8)
            tex1 = {k: torch.empty(W1 * H1 * 4, **u8) for k in TEX_ORDER[:6]}
            tex1['shN_centroids'] = torch.empty(cw1 * ch1 * 4, **u8)
            el1, meta1, _ = timed(lambda: ctx.dev_sog_sharded(comm1, tabs, args.iters, draws, tex1), ks, kw)
            sha1 = textures_digest(tex1, meta1)
            extras['sharded_world1'] = dict(record(workload(args, 1)[0] + ' through st_dev_sog_sharded (1-rank RCCL)',
                                                   total, el1, 'strong', sha1),
                                            textures_equal_main=sha1 == main_sha, parallelism='rowshard1-native')
            comm1.close()
            del tex1
            # the same shape with heavy-tailed correlated SH, 30% all-zero SH rows and clumped
            # positions: the assign's window on data like trained scenes, every label verified
            progress('extra record: realistic 10M')
            rt = realistic_table(total, SEED + 77, dev)
            rstep, rtex, _ = make_step([rt], total)
            el_r, meta_r, _ = timed(rstep, ks, kw)
            rstats = ctx.kmeans_stats() or None
            rver = None if args.no_verify else verify_step(ctx, rt, rtex, rstep, all_labels=not args.verify_sample)
            extras['realistic_10M'] = dict(
                record(f'writeSog SH3 of one {total / 1e6:g}M-splat table: heavy-tailed correlated SH (Student-t nu=3 '
                       'through a mixing matrix), 30% all-zero SH rows, 80% of the positions in 20,000 clumps; '
                       f'{args.iters} k-means iters', total, el_r, 'strong', textures_digest(rtex, meta_r)),
                vs_main_step=(el_r / ks) / (elapsed / args.steps), sh_kmeans_assign=rstats, verified=rver['ok'] if rver
                else None, verification=rver)
            del rt, rstep, rtex
            torch.cuda.empty_cache()
        # BASELINE config 4: one 50M-splat table, split over the ranks like the main table
        progress('extra record: config 4 (50M)')
        lo4, hi4 = CONFIG4_SPLATS * rank // world, CONFIG4_SPLATS * (rank + 1) // world
        t4 = [table_rows(CONFIG4_SPLATS, lo4, hi4, dev)]
        s4, tex4, _ = make_step(t4, CONFIG4_SPLATS)
        el4, meta4, _ = timed(s4, ks, kw)
        a4 = argparse.Namespace(**dict(vars(args), total_splats=CONFIG4_SPLATS))
        extras['config4_50M'] = record(workload(a4, world)[0], CONFIG4_SPLATS, el4, 'strong',
                                       textures_digest(tex4, meta4) if rank == 0 else None)
        del t4, s4, tex4
        torch.cuda.empty_cache()
        if world > 1:  # 10M splats per GPU (block `rank`): weak scaling
            progress('extra record: 10M splats per GPU')
            wt = [synth_table(10_000_000, SEED + rank, dev)]
            wstep, _, _ = make_step(wt, 10_000_000 * world)
            wel, _, _ = timed(wstep, ks, kw)
            aw = argparse.Namespace(**dict(vars(args), splats=10_000_000))
            extras['weak_10M_per_gpu'] = record(workload(aw, world)[0], 10_000_000 * world, wel, 'weak')
            del wt, wstep
            torch.cuda.empty_cache()

    if rank != 0:
        if comm:
            comm.close()
        if sharded:
            dist.destroy_process_group()
        if verification and not verification['ok']:
            sys.exit(1)
        return
    tex_sha = textures_digest(tex, meta)
    # the RCCL the library's collectives run on (st_rccl_info; the same file under the Node host)
    # and torch.distributed's own copy
    rccl_version = rccl_path = rccl_torch = None
    try:
        rccl_version, rccl_path = sh.rccl_info()
    except sh.StError as e:
        rccl_path = f'not loadable: {e}'
    try:
        rccl_torch = '.'.join(map(str, torch.cuda.nccl.version()))
    except Exception:
        pass
    # the .sog container of this step's textures on rank 0 (outside the headline's timed region)
    addr0, size0 = ctx.dev_sog_bundle_view(meta, total, tex, 0, 0)  # warm: workspace + pinned archive
    ref_archive = bytes((ctypes_char_array(size0)).from_address(addr0))
    ctx.set_profiling(True)
    ctx.reset_kernel_stats()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        _, archive_bytes = ctx.dev_sog_bundle_view(meta, total, tex, 0, 0)
    container_ms = (time.perf_counter() - t0) / args.steps * 1e3
    ckern = {}
    for name in ('webp.predict', 'webp.hist', 'webp.bits', 'webp.emit', 'crc32'):
        ms, cnt = ctx.kernel_stats(name)
        ckern[name] = ms / args.steps
    ctx.set_profiling(False)
    value = total * args.steps / elapsed / 1e6
    avg_sweep_s = (sweep_ms / max(sweep_launches, 1)) / 1e3
    D = 45
    flops_per_launch = 2.0 * n_local * pal * D  # nearest-centroid dot products, one assign pass (this rank)
    achieved = flops_per_launch / avg_sweep_s / 1e12 if sweep_launches else None
    e2e = None
    progress('end-to-end file run')
    if not sharded and not args.no_e2e:
        e2e = end_to_end(ctx, tabs[0], args.iters, draws, tex, ref_archive, meta)
    paths = None
    progress('config-3 stage table')
    if not sharded and not args.no_paths:
        # BASELINE config 3 (-r 0,45,0, filterNaN, Morton, chunk pack -> .compressed.ply) on its own
        # 10M SH-3 table: each HBM-bound stage priced by its algorithmic bytes (tools/bench_paths.py)
        sys.path.insert(0, os.path.join(ROOT, 'tools'))
        import bench_paths
        paths = bench_paths.measure(ctx, stream, dev, n=10_000_000, reps=5)
    progress('CPU baseline (oracle on the host cores)')
    cpu, cpu_all = (None, None) if (args.no_cpu_baseline or world > 1) else cpu_baseline(args)
    progress('writing the result')
    # HBM bytes per sweep launch from the committed rocprofv3 PMC passes (FETCH_SIZE x 2 + WRITE_SIZE
    # at this launch shape; tools/pmc_traffic.sh) -- PMC counters cannot be read from inside this run
    traffic, tsrc = None, None
    def latest(name):  # the newest round's committed profile of that name
        for rnd in ('r06', 'r05', 'r04', 'r03', 'r02', 'r01'):
            f = os.path.join(ROOT, 'profiles', rnd, name)
            if os.path.exists(f):
                return f
        return os.path.join(ROOT, 'profiles', 'r01', name)
    tfile = latest('pmc_sweep_traffic.json')
    if os.path.exists(tfile) and n_local == 10_000_000:
        traffic = json.load(open(tfile))['hbm_bytes_per_launch']
        tsrc = os.path.relpath(tfile, ROOT)
    # the engine clock the chip holds under the sweep (PMC GRBM_GUI_ACTIVE, tools/pmc.sh + pmc_util.py):
    # beside `frac` (against the 2.4 GHz headline peak), the fraction of the peak at that clock
    clock = None
    ufile = latest('pmc_sweep_util.json')
    if os.path.exists(ufile) and achieved:
        u = json.load(open(ufile))
        clock = {'engine_clock_GHz': u['engine_clock_GHz'], 'mfma_busy_frac': u['mfma_busy_frac'],
                 'peak_at_clock': u['dense_fp16_peak_at_this_clock_TFLOPs'],
                 'frac_at_clock': achieved / u['dense_fp16_peak_at_this_clock_TFLOPs'],
                 'source': os.path.relpath(ufile, ROOT)}
    out = {
        'metric': 'Msplats/sec PLY->SOG (SH-3, 10 k-means iters)',
        'headline': ('device pipeline, resident table (PLY ingest and WebP/ZIP excluded; see end_to_end_file '
                     'for the PLY file -> .sog file job, end_to_end_file.node_host for the Node drop-in)'),
        'value': value,
        'unit': 'Msplats/s',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': elapsed / args.steps * 1e3,
        'higher_is_better': True,
        'scaling': scaling,
        'vs_baseline': None,
        'dtype': 'f64+f32 (bit-exact JS semantics); fp16 MFMA (f32 accumulate) for the assign prefilter',
        'data': 'synthetic (SURVEY.md 8d distributions, torch Generator seeds 1002+rank / 5001+file), resident in HBM',
        'config': {'workload': wl_desc, 'splats_total': total, 'splats_rank0': n_local, 'sh_bands': 3,
                   'palette_size': pal, 'iterations': args.iters,
                   'parallelism': (f'rowshard{world}' + ('-pytorch' if args.dist_python else '-native'))
                   if sharded else 'single'},
        'roofline': {
            'kernel': 'k_sweep<KS=3> (v_mfma_f32_32x32x16_f16 nearest-centroid score |c|^2-2p.c, top-3 tile minima per splat)',
            'bound': 'mfma',
            'achieved': achieved,
            'peak': MFMA_F16_DENSE_TFLOPS,
            'unit': 'TFLOP/s',
            'frac': (achieved / MFMA_F16_DENSE_TFLOPS) if achieved else None,
            'traffic': traffic,
            'traffic_unit': 'bytes per launch',
            'traffic_source': tsrc,
            'algorithmic_flops_per_launch': flops_per_launch,
            'avg_launch_ms': avg_sweep_s * 1e3,
            'launches': sweep_launches,
            'clock': clock,
        },
        'cpu_baseline': cpu,
        'cpu_baseline_all_cores': cpu_all,
        'container': {
            'what': 'st_dev_sog_bundle_view: WebP lossless x7 + CRC-32 + ZIP of this step\'s textures, archive in '
                    'pinned host memory (rank 0)',
            'ms': container_ms,
            'archive_bytes': archive_bytes,
            'kernel_ms': ckern,
            'end_to_end_ms_per_step': elapsed / args.steps * 1e3 + container_ms,
            'end_to_end_Msplats_per_s': total / (elapsed / args.steps + container_ms / 1e3) / 1e6,
        },
        'end_to_end_file': e2e,
        'paths_config3': paths,
        'stages_ms': stages,
        'sog_stages': sog_stage_table(stages, n_local, args.iters),
        'kernels': kstats,
        'draws_used_per_step': used,
        'sh_kmeans_assign': sh_assign,
        'rccl_ranks': rccl_ranks,
        'rccl_version': rccl_version,
        'rccl_path': rccl_path,
        'rccl_torch_version': rccl_torch,
        'torch_backend': torch_backend(args) if sharded else None,
        'transport': transport,
        'side_channel': (os.environ.get('ST_SIDE_CHANNEL') != '0') if comm else None,
        'distinct_devices': devices if sharded else 1,
        'textures_sha256': tex_sha,
        'extra_records': extras or None,
        'verified': verification['ok'] if verification else None,
        'verification': verification,
    }
    _RESULT.write(json.dumps(out) + '\n')
    _RESULT.flush()
    if comm:
        comm.close()
    if sharded:
        dist.destroy_process_group()
    if verification and not verification['ok']:
        sys.exit(1)


# stdout carries exactly the one JSON line: whatever the libraries print there (RCCL's
# version banner, for one) goes to stderr instead
_RESULT = sys.stdout

if __name__ == '__main__':
    _args = parse()
    sys.stdout.flush()
    _RESULT = os.fdopen(os.dup(1), 'w')
    os.dup2(2, 1)
    sys.stdout = sys.stderr
    if _args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        sys.exit(launch(_args, sys.argv[1:]))
    if 'WORLD_SIZE' in os.environ and int(os.environ['WORLD_SIZE']) != _args.gpus and _args.gpus != 1:
        raise SystemExit(f'bench.py: --gpus {_args.gpus} under a launcher of WORLD_SIZE={os.environ["WORLD_SIZE"]}')
    main(_args)
