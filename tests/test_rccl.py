"""The RCCL exchange paths of killerbeez_amd.dist executed on the GPU: a
one-rank `nccl` process group (RCCL on ROCm) with every all-gather forced, so the sharded
triage, the merger fold (merger/merger.c:79-104) and the unique crash/hang table go through
RCCL collectives on real device buffers on a one-GPU box.  The results must equal one
sequential pass (the CPU oracle, the plain AND, insert-if-absent in trace order).  Unmeasured
for N > 1: the driver's node run exercises more ranks."""
import socket

import numpy as np
import pytest

import oracle
from killerbeez_amd import synth
from killerbeez_amd.triage import WANT_H32, TriageContext, UniqueSet

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def nccl_world1(gpu):
    import torch.distributed as dist

    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0,
                            world_size=1, device_id=gpu)
    assert dist.get_backend() == "nccl"
    yield gpu
    dist.destroy_process_group()


def _rccl_mapped():
    with open("/proc/self/maps") as f:
        return any("librccl" in line for line in f)


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_triage_sharded_over_rccl(nccl_world1, mode):
    import torch

    from killerbeez_amd.dist import triage_sharded

    m, n = 4096, 900
    v = np.full((3, m), 0xFF, np.uint8)
    last = 0
    with TriageContext(m, mode, n) as ctx:
        for batch in range(3):
            t, oc = synth.sparse_np(n, m, seed=40 + batch, hot_frac=0.05)
            t[200] = t[199]
            exp = oracle.triage_batch(mode, t, oc, virgin=v, last_hash=last, want=oracle.WANT_H32)
            out = triage_sharded(ctx, torch.from_numpy(t).cuda(), torch.from_numpy(oc).cuda(),
                                 [n], 0, 1, WANT_H32, device=nccl_world1, force_collective=True)
            torch.cuda.synchronize()
            ctx.sync()
            np.testing.assert_array_equal(out["hnb"].cpu().numpy(), exp["hnb"])
            np.testing.assert_array_equal(out["h32"].cpu().numpy().view(np.uint32), exp["h32"])
            np.testing.assert_array_equal(ctx.get_virgin(), exp["virgin"])
            if mode == 1:
                assert ctx.last_hash == exp["last_hash"]
            v, last = exp["virgin"], exp.get("last_hash", 0)
    assert _rccl_mapped()


def test_merge_sharded_over_rccl(nccl_world1):
    import torch

    from killerbeez_amd.dist import merge_sharded

    rng = np.random.default_rng(3)
    st = np.full((2500, 3 * 65536), 0xFF, np.uint8)
    clear = rng.random(st.shape) < 0.002
    st[clear] = rng.integers(0, 255, int(clear.sum()), dtype=np.uint8)
    got = merge_sharded(torch.from_numpy(st).cuda(), 1, force_collective=True)
    np.testing.assert_array_equal(got.cpu().numpy(), np.bitwise_and.reduce(st, axis=0))


def test_dedup_sharded_over_rccl(nccl_world1):
    """Two batches into one replica: the first with a fixed cap, the second negotiating it with
    an RCCL all_reduce(MAX)."""
    import torch

    from killerbeez_amd.dist import dedup_sharded

    rng = np.random.default_rng(4)
    table = UniqueSet(1 << 12)
    seen = set()
    for b, cap in enumerate((1000, None)):
        k = np.stack([rng.integers(0, 300, 1000), rng.integers(1, 3, 1000)], 1).astype(np.int64)
        mask = rng.random(1000) < 0.7
        exp = np.zeros(1000, np.uint8)
        for j in range(1000):
            key = (int(k[j, 0]), int(k[j, 1]))
            if mask[j] and key not in seen:
                seen.add(key)
                exp[j] = 1
        got = dedup_sharded(table, torch.from_numpy(k).cuda(), torch.from_numpy(mask).cuda(), 0, 1,
                            cap=cap, force_collective=True)
        np.testing.assert_array_equal(got.cpu().numpy(), exp)
    assert table.size() == len(seen)
