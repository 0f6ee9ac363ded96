"""The N>1 path on CPU: world_size-2 gloo ranks, as bench.py runs them under
torchrun (one process per GPU, RCCL).  Each rank runs the library's host
side of the pipeline on its own shard -- packed lowering (dp_lower_into),
chunk planning and staging (dp_stage_roundtrip), result stitching
(dp_stitch_selftest), the device partition (dp_partition) -- and the oracle
stands in for the device solve, so sharding, the host path per rank and the
timing reduction are checked here.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from deppy_amd import _lib, shard

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

N_PER_RANK = 40


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _lowered(config, n, seed, packed=False):
    w = _lib.generate(config, n, seed)
    wa = _lib.WireArrays(**{k: w[k] for k in (
        "prob_var_off", "var_id", "var_con_off", "con_kind", "con_n", "con_arg_off", "con_arg",
        "str_off")}, str_bytes=w["str_bytes"].tobytes())
    return _lib.Lowered(wa, narrow=packed, packed=packed)


def _host_path(seed, n):
    """The library's host side of dp_submit on one shard: packed records,
    their chunked staging round trip, stitched synthetic results, the
    partition over 2 devices."""
    lwp = _lowered(2, n, seed, packed=True)
    staged, firsts = _lib.stage_roundtrip(lwp.rec_off, lwp.rec, 0, chunk_problems=16)
    st = _lib.stitch_selftest(lwp.rec_off, lwp.rec, 16)
    cut = _lib.partition(lwp.rec_off, 2)
    return dict(prec=lwp.rec.copy(), prec_off=lwp.rec_off.copy(), staged=staged, firsts=firsts,
                st_status=st["status"][:n], st_installed=st["installed"], st_core=st["core"],
                st_core_len=st["core_len"][:n], cut=cut)


def _rank(rank, world, port, outdir):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from oracle import oracle
    g = shard.init_from_env("gloo")
    seed = shard.shard_seed(7, g.rank, N_PER_RANK)
    lw = _lowered(2, N_PER_RANK, seed)
    res = oracle.solve_batch(lw.rec_off, lw.rec, 0, 1)
    host = _host_path(seed, N_PER_RANK)
    # the packed records solve like the int32 ones (oracle reads every form)
    pres = oracle.solve_batch(host["prec_off"], host["prec"], 0, 1)
    assert np.array_equal(pres["status"], res["status"]) and np.array_equal(pres["steps"], res["steps"])
    g.barrier()
    fake_elapsed = 1.0 + g.rank  # rank 1 is the slowest
    mx = g.max(fake_elapsed)
    all_t = g.gather(fake_elapsed)
    np.savez(os.path.join(outdir, "r%d.npz" % g.rank), rec_off=lw.rec_off, rec=lw.rec,
             status=res["status"], steps=res["steps"], installed=res["installed"],
             mx=mx, all_t=np.array(all_t), **{"host_" + k: v for k, v in host.items()})
    g.close()


def test_shard_seed_slices_one_global_sequence():
    assert shard.shard_seed(1000, 0, 10000) == 1000
    assert shard.shard_seed(1000, 3, 10000) == 31000
    assert shard.aggregate_rate(10000, 8, 20, 2.0) == 8 * 10000 * 20 / 2.0


def test_single_rank_group_is_local():
    g = shard.Group()
    g.barrier()
    assert g.max(3.5) == 3.5 and g.gather(2.0) == [2.0]


@pytest.mark.timeout(300)
def test_two_rank_gloo(tmp_path):
    from oracle import oracle
    port = _free_port()
    mp.start_processes(_rank, args=(2, port, str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    r = [np.load(tmp_path / ("r%d.npz" % i)) for i in range(2)]
    # timing reduction: every rank sees the max and the full gather
    for x in r:
        assert float(x["mx"]) == 2.0
        assert list(x["all_t"]) == [1.0, 2.0]
    # the two shards are the two halves of the single-process global batch
    glob = _lowered(2, 2 * N_PER_RANK, 7)
    gres = oracle.solve_batch(glob.rec_off, glob.rec, 0, 2)
    ro = glob.rec_off
    half = int(ro[N_PER_RANK])
    assert np.array_equal(r[0]["rec"], glob.rec[:half])
    assert np.array_equal(r[1]["rec"], glob.rec[half:])
    assert np.array_equal(np.concatenate([r[0]["status"], r[1]["status"]]), gres["status"])
    assert np.array_equal(np.concatenate([r[0]["steps"], r[1]["steps"]]), gres["steps"])
    # no two ranks solved the same catalog
    assert not np.array_equal(r[0]["rec"], r[1]["rec"])
    # each rank's host path equals the same path run here on that rank's shard
    for i in range(2):
        want = _host_path(7 + i * N_PER_RANK, N_PER_RANK)
        for k, v in want.items():
            assert np.array_equal(r[i]["host_" + k], v), (i, k)
        # staging round trip: packed one-wavefront records are staged as they are
        assert np.array_equal(r[i]["host_staged"], r[i]["host_prec"])
        assert list(r[i]["host_firsts"]) == list(range(0, N_PER_RANK, 16))


def test_strong_scaling_ranges_partition_the_total():
    """bench.py --scaling strong: the ranks' contiguous shares cover the
    config's total exactly once (config 3: 1M catalogs over 1/2/4/8 GPUs)."""
    from deppy_amd import shard
    for total in (1_000_000, 10_001, 7):
        for world in (1, 2, 4, 8):
            rs = [shard.strong_range(total, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            assert max(h - l for l, h in rs) - min(h - l for l, h in rs) <= 1


def test_bench_refuses_world_mismatch(monkeypatch):
    """bench.py --gpus N must run on N ranks: under a launcher with another
    WORLD_SIZE it stops instead of measuring something else."""
    import subprocess
    import sys
    env = dict(__import__("os").environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE" in (r.stderr + r.stdout)
