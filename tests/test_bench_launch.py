"""bench.py's multi-GPU launch contract.

CPU: `python bench.py --gpus N` with no launcher around it starts the N-rank job itself (a child
torch.distributed.run) without importing torch in the parent, relays rank 0's JSON line and fails
unless the job reports N ranks; the synthetic tables are fixed-seed blocks sliced by global row
range, so a T-splat table does not depend on how many ranks split it.

GPU: the self-launched 2-rank rehearsal on one GPU (--backend gloo: the library's own sharded
path, st_dev_sog_sharded in two processes over its host shared-memory transport) prints n_gpus 2
and the same textures_sha256 as one GPU over the same table."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, 'bench.py')
sys.path.insert(0, ROOT)


def test_launcher_command_and_parent_never_imports_torch():
    r = subprocess.run([sys.executable, BENCH, '--gpus', '8', '--steps', '20', '--warmup', '5', '--launch-dry-run'],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    cmd = out['cmd']
    assert out['torch_imported'] is False
    assert cmd[1:3] == ['-m', 'torch.distributed.run']
    assert '--nproc-per-node=8' in cmd and '--nnodes=1' in cmd and '--master-addr=127.0.0.1' in cmd
    i = cmd.index(BENCH)
    assert cmd[i + 1:i + 7] == ['--gpus', '8', '--steps', '20', '--warmup', '5']


def _fake_job(tmp_path, n_reported, rc=0):
    script = tmp_path / 'job.py'
    script.write_text('import json, sys\n'
                      'print("rank chatter")\n'
                      f'print(json.dumps({{"metric": "m", "value": 1.0, "n_gpus": {n_reported}}}))\n'
                      f'sys.exit({rc})\n')
    return [sys.executable, str(script)]


@pytest.mark.parametrize('reported,rc,want_rc', [(4, 0, 0), (1, 0, 3), (4, 7, 7)])
def test_launch_relays_rank0_line_and_checks_world(tmp_path, reported, rc, want_rc):
    """the parent relays exactly the result line; a job that ran the wrong number of ranks or
    failed makes the parent fail"""
    code = ('import sys, io, json; sys.path.insert(0, %r); import bench; '
            'bench.launcher_cmd = lambda argv, n, port: %r; '
            'bench._RESULT = sys.stdout; sys.stdout = sys.stderr; '
            'a = bench.parse(["--gpus", "4"]); rc = bench.launch(a, ["--gpus", "4"]); '
            'assert "torch" not in sys.modules; sys.exit(rc)') % (ROOT, _fake_job(tmp_path, reported, rc))
    r = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True, timeout=120)
    assert r.returncode == want_rc, r.stderr
    if want_rc == 0:
        lines = r.stdout.strip().splitlines()
        assert len(lines) == 1 and json.loads(lines[0])['n_gpus'] == 4
        assert 'rank chatter' in r.stderr


def _launch(tmp_path, script_text, extra=()):
    script = tmp_path / 'job.py'
    script.write_text(script_text)
    code = ('import sys, io, json; sys.path.insert(0, %r); import bench; '
            'bench.launcher_cmd = lambda argv, n, port: %r; '
            'bench._RESULT = sys.stdout; sys.stdout = sys.stderr; '
            'a = bench.parse(["--gpus", "2"] + %r); rc = bench.launch(a, ["--gpus", "2"]); '
            'assert "torch" not in sys.modules; sys.exit(rc)') % (ROOT, [sys.executable, str(script)], list(extra))
    return subprocess.run([sys.executable, '-c', code], capture_output=True, text=True, timeout=120)


def test_launch_kills_a_stalled_job_and_reruns_without_side_channel(tmp_path):
    """a job whose progress lines stop is killed (its process group) after --launch-stall seconds
    and rerun once with ST_SIDE_CHANNEL=0; the relayed line says so"""
    r = _launch(tmp_path, 'import json, os, sys, time\n'
                          'print("@@progress rank=0 started", flush=True)\n'
                          'if os.environ.get("ST_SIDE_CHANNEL") != "0":\n'
                          '    time.sleep(60)\n'
                          'print(json.dumps({"metric": "m", "value": 1.0, "n_gpus": 2}))\n',
                ['--launch-stall', '2'])
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out['fallback']['side_channel'] == 'off' and 'no progress' in out['fallback']['first_job']
    assert 'killing the job' in r.stderr


def test_launch_budget_and_a_failing_fallback(tmp_path):
    """a job that keeps reporting progress but never finishes hits --launch-budget; when the rerun
    fails too the parent exits non-zero"""
    r = _launch(tmp_path, 'import time\n'
                          'for i in range(100):\n'
                          '    print("@@progress rank=0 step", i, flush=True)\n'
                          '    time.sleep(0.5)\n',
                ['--launch-budget', '3', '--launch-stall', '30'])
    assert r.returncode != 0
    assert r.stderr.count('killing the job') == 2 and 'budget' in r.stderr


def test_workload_is_the_same_at_every_n():
    """the default run is north_star's workload -- one 10M-splat table, strong-scaled -- at every N,
    so the driver's 1/2/4/8-GPU values divide the same job; config 4 and config 5 likewise"""
    import bench
    for extra in ([], ['--total-splats', '50000000'], ['--merge', '4']):
        rec = {}
        for n, backend in ((1, 'nccl'), (2, 'gloo'), (2, 'nccl'), (4, 'nccl'), (8, 'nccl')):
            a = bench.parse(['--gpus', str(n), '--backend', backend] + extra)
            rec[(n, backend)] = bench.workload(a, n)
        assert len(set(rec.values())) == 1, rec
        desc, total, scaling = rec[(1, 'nccl')]
        assert scaling == 'strong'
        if not extra:
            assert total == 10_000_000 and desc.startswith('north_star: ')
    # weak scaling (--splats S per GPU): same description, S x N splats
    w1 = bench.workload(bench.parse(['--splats', '10000000']), 1)
    w8 = bench.workload(bench.parse(['--gpus', '8', '--splats', '10000000']), 8)
    assert w1[0] == w8[0] and (w1[1], w8[1]) == (10_000_000, 80_000_000) and w8[2] == 'weak'


def test_torch_process_group_is_gloo_beside_the_librarys_rccl():
    """torch.distributed only serves bench.py between steps (barriers, the unique id, the timer, the
    verification), so it runs on gloo and each rank initialises one RCCL: the library's
    (st_rccl.cpp).  The torch harness (--dist-python) steps through torch collectives: its backend."""
    import bench
    for argv in (['--gpus', '8'], ['--gpus', '8', '--backend', 'gloo'], ['--dist'], ['--gpus', '2', '--merge', '4']):
        assert bench.torch_backend(bench.parse(argv)) == 'gloo', argv
    assert bench.torch_backend(bench.parse(['--gpus', '2', '--dist-python'])) == 'nccl'
    assert bench.torch_backend(bench.parse(['--gpus', '2', '--dist-python', '--backend', 'gloo'])) == 'gloo'
    assert bench.torch_backend(bench.parse(['--gpus', '8', '--torch-backend', 'nccl'])) == 'nccl'


def test_table_rows_independent_of_the_split():
    """rows [lo, hi) of a T-row table built from fixed-seed blocks: any split concatenates to the
    same table (small blocks here; the bench uses 10M-row blocks)"""
    import torch

    import bench
    T, blk = 2_500, 1_000
    whole = bench.table_rows(T, 0, T, 'cpu', block=blk)
    for cuts in ([0, 700, 2_500], [0, 1_000, 2_000, 2_500], [0, 0, 1_250, 2_499, 2_500]):
        parts = [bench.table_rows(T, a, b, 'cpu', block=blk) for a, b in zip(cuts, cuts[1:])]
        for k in whole:
            assert torch.equal(torch.cat([p[k] for p in parts]), whole[k]), (cuts, k)
    # 10M-per-GPU weak scaling: rank r's rows are block r (seed 1002 + r)
    blk0 = bench.synth_table(1_000, bench.SEED + 1, 'cpu')
    r1 = bench.table_rows(3_000, 1_000, 2_000, 'cpu', block=1_000)
    assert all(torch.equal(blk0[k], r1[k]) for k in blk0)


@pytest.mark.gpu
def test_self_launched_two_ranks_match_one_gpu(tmp_path):
    """`bench.py --gpus 2 --backend gloo` (no torchrun on the command line) rehearsed on one GPU:
    two processes running the library's st_dev_sog_sharded over its host shared-memory transport,
    and the textures of the 4M-splat table equal one GPU's"""
    common = ['--steps', '1', '--warmup', '0', '--no-cpu-baseline', '--no-e2e', '--no-paths']
    env = dict(os.environ, PYTHONUNBUFFERED='1')
    r2 = subprocess.run([sys.executable, BENCH, '--gpus', '2', '--backend', 'gloo', '--no-weak',
                         '--splats', '2000000'] + common, capture_output=True, text=True, timeout=600, env=env)
    assert r2.returncode == 0, r2.stderr[-4000:]
    two = json.loads(r2.stdout.strip().splitlines()[-1])
    assert two['config']['parallelism'] == 'rowshard2-native' and two['transport'] == 'host-shm'
    assert 'fallback' not in two
    # each rank checked every label of its shard against the reference's definitions
    assert two['verified'] and two['verification']['labels_checked'] == 4_000_000, two['verification']
    assert two['verification']['centroids_identical_on_every_rank']
    r1 = subprocess.run([sys.executable, BENCH, '--gpus', '1', '--splats', '4000000'] + common + ['--no-verify'],
                        capture_output=True, text=True, timeout=600, env=env)
    assert r1.returncode == 0, r1.stderr[-4000:]
    one = json.loads(r1.stdout.strip().splitlines()[-1])
    assert two['n_gpus'] == 2 and two['distinct_devices'] == 1 and one['n_gpus'] == 1
    assert two['config']['splats_total'] == one['config']['splats_total'] == 4_000_000
    assert two['textures_sha256'] == one['textures_sha256']
