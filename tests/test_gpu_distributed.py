"""GPU: the multi-GPU path's collectives on the device backend. One process group of size 1 over
``nccl`` (RCCL) on cuda:0, in a child process: the setup broadcast (``distributed.broadcast_arrays``:
size, header and payload broadcasts of device tensors), the counter all-reduces and the BER sweep's
per-round error exchange (``ber._dist_exchange``: an all-reduce of a device tensor) all run through
RCCL — a size-1 group still executes every collective — and give the results of the undistributed
run. (A multi-rank RCCL run needs one GPU per rank; the 8-GPU node is the driver's. The multi-rank
logic is covered with gloo, world size 2, in tests/test_cpu_distributed.py / test_cpu_channel.py.)"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = r"""
import json, os, sys
import numpy as np
import torch
import torch.distributed as dist
sys.path.insert(0, os.environ["IBL_ROOT"])
from informationbottleneckdecodingldpc_amd import codes, distributed, graph, tables
from informationbottleneckdecodingldpc_amd.ber import BERConfig, run_ber
from informationbottleneckdecodingldpc_amd.discrete_LDPC_decoder_irreg import Discrete_LDPC_Decoder_class_irregular
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
try:
    assert dist.get_backend() == "nccl"
    g = graph.build_graph(codes.wlan_80211n())
    tb = tables.random_tables(16, 16, g.d_c_max, g.d_v_max, 5, seed=3)
    arrays = dict(indptr=g.csr_indptr, cols=g.csr_cols, cn=tb.cn, small=np.arange(7, dtype=np.int16))
    got = distributed.broadcast_arrays(arrays, src=0)
    same = all(np.array_equal(got[k], arrays[k]) and got[k].dtype == arrays[k].dtype for k in arrays)
    tot = distributed.allreduce_counts({"errors": 5, "codewords": 7})
    mx = distributed.allreduce_max(2.5)
    cfg = BERConfig(**json.loads(os.environ["IBL_CFG"]))
    H = codes.wlan_80211n()
    tl = tables.llr_tables(np.linspace(-6, 6, 16), g.d_c_max, g.d_v_max, 10)
    dec = Discrete_LDPC_Decoder_class_irregular(H, 10, 16, 16, tl.cn, tl.vn, tl.match_cn, tl.match_vn,
                                                cfg.msg_at_time, match="true")
    r = run_ber(dec, cfg)
    print("RESULT " + json.dumps({"same": bool(same), "tot": tot, "mx": mx, "errors": [float(e) for e in r.errors],
                                  "blocks": list(r.blocks), "ebn0": [float(x) for x in r.EbN0_dB_vector]}))
finally:
    dist.destroy_process_group()
"""


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_group_collectives_and_ber_exchange():
    from informationbottleneckdecodingldpc_amd import codes, graph, tables
    from informationbottleneckdecodingldpc_amd.ber import BERConfig, run_ber
    from informationbottleneckdecodingldpc_amd.discrete_LDPC_decoder_irreg import \
        Discrete_LDPC_Decoder_class_irregular
    cfg = dict(EbN0_dB_start=1.0, EbN0_dB_max_value=2.0, EbN0_dB_normal_stepwidth=1.0, EbN0_dB_small_stepwidth=0.5,
               target_error_rate=1e-9, min_errors=3000, msg_at_time=64, max_blocks=256, seed=4, sync_every=2)
    env = dict(os.environ, IBL_ROOT=ROOT, IBL_CFG=json.dumps(cfg), MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, "-c", _CHILD], env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")][-1]
    res = json.loads(line[len("RESULT "):])
    assert res["same"] and res["tot"] == {"codewords": 7, "errors": 5} and res["mx"] == 2.5
    # the same sweep without a process group, in this process
    H = codes.wlan_80211n()
    g = graph.build_graph(H)
    tl = tables.llr_tables(np.linspace(-6, 6, 16), g.d_c_max, g.d_v_max, 10)
    dec = Discrete_LDPC_Decoder_class_irregular(H, 10, 16, 16, tl.cn, tl.vn, tl.match_cn, tl.match_vn, 64,
                                                match="true")
    r = run_ber(dec, BERConfig(**cfg))
    assert res["errors"] == [float(e) for e in r.errors] and res["blocks"] == list(r.blocks)
    assert len(res["ebn0"]) == 2
    torch.cuda.synchronize()


def test_c_abi_communicator_size_one():
    """The C ABI's RCCL communicator (ibl_comm_*: for callers without torch.distributed) as a 1-rank group on the
    box's GPU: the setup broadcast leaves the root's bytes in place, the counter all-reduce sums over one rank."""
    import ctypes

    import torch
    from informationbottleneckdecodingldpc_amd import _lib
    L = _lib.load()
    uid = (ctypes.c_uint8 * _lib.IBL_COMM_ID_BYTES)()
    _lib.check(L.ibl_comm_unique_id(uid), "ibl_comm_unique_id")
    comm = ctypes.c_void_p()
    _lib.check(L.ibl_comm_create(uid, 1, 0, 0, ctypes.byref(comm)), "ibl_comm_create")
    try:
        s = torch.cuda.current_stream().cuda_stream
        buf = torch.arange(1000, dtype=torch.uint8, device="cuda:0")
        want = buf.clone()
        _lib.check(L.ibl_comm_broadcast(comm, buf.data_ptr(), buf.numel(), 0, s), "ibl_comm_broadcast")
        cnt = torch.tensor([5, -3, 2 ** 40], dtype=torch.int64, device="cuda:0")
        _lib.check(L.ibl_comm_allreduce_sum_i64(comm, cnt.data_ptr(), 3, s), "ibl_comm_allreduce_sum_i64")
        torch.cuda.synchronize()
        assert torch.equal(buf, want)
        assert cnt.cpu().tolist() == [5, -3, 2 ** 40]
        with pytest.raises(_lib.IBLError):
            _lib.check(L.ibl_comm_broadcast(comm, buf.data_ptr(), 10, 1, s), "ibl_comm_broadcast")   # root >= nranks
    finally:
        L.ibl_comm_destroy(comm)
