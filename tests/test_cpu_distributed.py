"""CPU: the multi-GPU path's host logic over torch.distributed with gloo, world_size 2:
setup broadcast of graph + tables from rank 0, disjoint codeword shards, counter all-reduce."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from informationbottleneckdecodingldpc_amd.distributed import shard_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist

    from informationbottleneckdecodingldpc_amd import codes, distributed, graph, tables
    rank_, world_, _ = distributed.init_from_env(backend="gloo")
    try:
        if rank_ == 0:
            g = graph.build_graph(codes.wlan_80211n())
            tb = tables.random_tables(16, 16, g.d_c_max, g.d_v_max, 5, seed=3)
            arrays = dict(indptr=g.csr_indptr, cols=g.csr_cols, cn=tb.cn, vn=tb.vn, mc=tb.match_cn,
                          rate=np.array([g.R_c]), small=np.arange(7, dtype=np.int16))
        else:
            arrays = None
        got = distributed.broadcast_arrays(arrays, src=0)
        start, count = distributed.shard_range(1000, rank_, world_)
        tot = distributed.allreduce_counts({"errors": rank_ + 1, "codewords": count})
        mx = distributed.allreduce_max(float(rank_) * 2.5)
        digest = {k: (v.dtype.str, v.shape, float(np.asarray(v, dtype=np.float64).sum())) for k, v in got.items()}
        q.put((rank_, digest, start, count, tot, mx))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_broadcast_shard_allreduce():
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    (r0, d0, s0, c0, t0, m0), (r1, d1, s1, c1, t1, m1) = res
    assert d0 == d1 and set(d0) == {"indptr", "cols", "cn", "vn", "mc", "rate", "small"}
    assert d0["small"][0] == "<i2" and d0["small"][1] == (7,)
    assert (s0, c0, s1, c1) == (0, 500, 500, 500)
    assert t0 == t1 == {"codewords": 1000, "errors": 3}
    assert m0 == m1 == 2.5


def _bench_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist

    import bench
    from informationbottleneckdecodingldpc_amd import distributed
    distributed.init_from_env(backend="gloo")
    try:
        q.put((rank, bench.aggregate_rate(1000, 4, 2.0 if rank == 0 else 4.0)))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_bench_aggregation():
    """bench.py's whole-job rate: world·B·steps ÷ the slowest rank's time, and the record names the backend,
    the world size and the per-rank rates."""
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bench_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == res[1]
    r = res[0]
    assert r["value"] == 2 * 1000 * 4 / 4.0 and r["elapsed_max_s"] == 4.0
    assert r["world_size"] == 2 and r["backend"] == "gloo"
    assert r["per_rank_codewords_per_s"] == {"min": 1000.0, "max": 2000.0}


def test_gloo_refused_with_one_gpu_per_rank(monkeypatch):
    import torch

    from informationbottleneckdecodingldpc_amd import distributed
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.delenv("IBL_SHARE_DEVICE", raising=False)
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "set_device", lambda d: None)
    with pytest.raises(RuntimeError, match="refusing the gloo backend"):
        distributed.init_from_env(backend="gloo")


@pytest.mark.parametrize("total,world", [(64 * 1024, 8), (10, 3), (7, 8), (0, 2)])
def test_shard_range_partitions(total, world):
    spans = [shard_range(total, r, world) for r in range(world)]
    assert sum(c for _, c in spans) == total
    pos = 0
    for s, c in spans:
        assert s == pos
        pos += c
    assert max(c for _, c in spans) - min(c for _, c in spans) <= 1


@pytest.mark.parametrize("total,world", [(0, 1), (7, 3), (8192, 8), (65536, 8), (100, 7), (5, 8)])
def test_c_abi_shard_range_equals_python(total, world):
    """ibl_shard_range (the batch split for callers without torch, include/ibldpc.h) equals distributed.shard_range:
    contiguous ranges that tile [0, total) with sizes differing by at most one."""
    from informationbottleneckdecodingldpc_amd import _lib
    from informationbottleneckdecodingldpc_amd.distributed import shard_range
    got = [_lib.shard_range(total, r, world) for r in range(world)]
    assert got == [shard_range(total, r, world) for r in range(world)]
    assert sum(c for _, c in got) == total and all(got[r][0] + got[r][1] == got[r + 1][0] for r in range(world - 1))
    with pytest.raises(_lib.IBLError):
        _lib.shard_range(total, world, world)
