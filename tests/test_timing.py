"""The diagnostics timers (kbz_ctx_time_pass1 / kbz_ctx_time_stages) with timing left on for more
batches than their event pools hold: the oldest records are folded into running sums, nothing is
lost and nothing grows without bound (the pool grew two events per stage per batch)."""
import numpy as np
import pytest
import torch

from killerbeez_amd import synth
from killerbeez_amd.triage import MODE_DYNAMORIO, WANT_H32, TriageContext

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("staged", [False, True], ids=["fused", "staged"])
def test_timers_fold_past_pool(gpu, staged, monkeypatch):
    if staged:
        monkeypatch.setenv("KBZ_DEBUG_STAGED", "1")
    m, n, k = 4096, 128, 1200  # 1,200 batches: past the 512-record fold point twice
    t, oc = synth.sparse_torch(n, m, device="cuda")
    with TriageContext(m, MODE_DYNAMORIO, n) as ctx:
        ctx.time_pass1(True)
        ctx.time_stages(True)
        for _ in range(k):
            ctx.triage(t, oc, WANT_H32)
        torch.cuda.synchronize()
        ms, launches = ctx.time_pass1(False)
        st, nb = ctx.time_stages(False)
        assert launches == k and ms > 0
        assert nb == k
        assert all(np.isfinite(v) and v >= 0 for v in st.values()) and st["scan"] > 0
        # reading resets both
        assert ctx.time_pass1(False) == (0.0, 0)
        assert ctx.time_stages(False)[1] == 0


def test_time_one_launch_in_every(gpu):
    """kbz_ctx_time_pass1_every: 10 batches timed one in 4 -> launches 0, 4 and 8."""
    m, n = 4096, 128
    t, oc = synth.sparse_torch(n, m, device="cuda")
    with TriageContext(m, MODE_DYNAMORIO, n) as ctx:
        ctx.time_pass1_every(4)
        ctx.time_pass1(True)
        for _ in range(10):
            ctx.triage(t, oc, WANT_H32)
        torch.cuda.synchronize()
        ms, launches = ctx.time_pass1(False)
        assert launches == 3 and ms > 0
        ctx.time_pass1_every(1)
        ctx.time_pass1(True)
        for _ in range(5):
            ctx.triage(t, oc, WANT_H32)
        torch.cuda.synchronize()
        assert ctx.time_pass1(False)[1] == 5
