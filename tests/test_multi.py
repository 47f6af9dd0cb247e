"""The merger fold sharded over GPUs from C (kbz_merge_and_fill_devices, include/kbz_triage.h):
merger/merger.c:79-104 with the states split across workers, one per GPU (several may share a
GPU), exchanged by copies or RCCL and ANDed.  On a one-GPU box the workers share cuda:0 and the
copy path runs, and the RCCL path runs as a one-rank communicator (devices=[0]); the RCCL
all-gather between distinct GPUs is exercised only where the box has two or more (unmeasured
on the one-GPU box: its results are the same AND)."""
import os

import numpy as np
import pytest

from killerbeez_amd import plugin as P
from killerbeez_amd.triage import EXCHANGE_COPY, EXCHANGE_RCCL, merge_and_devices


def _states(n, nbytes, seed):
    rng = np.random.default_rng(seed)
    st = np.full((n, nbytes), 0xFF, np.uint8)
    clear = rng.random((n, nbytes)) < 0.003
    st[clear] = rng.integers(0, 255, int(clear.sum()), dtype=np.uint8)
    return st


@pytest.mark.gpu
@pytest.mark.parametrize("workers", [1, 2, 3, 8])
def test_merge_devices_copy_path(gpu, workers):
    st = _states(1000, 3 * 4096, 11 + workers)
    out, used = merge_and_devices(st, devices=[0] * workers)
    assert used == EXCHANGE_COPY
    np.testing.assert_array_equal(out, np.bitwise_and.reduce(st, axis=0))


@pytest.mark.gpu
def test_merge_devices_golden_and_edges(gpu):
    """The reference-built golden merge (tests/golden/merge.npz: 5 states of 3 maps through the
    reference's afl_merge), fewer states than workers, odd state sizes, no state."""
    from tests.test_golden import _merge_fixture

    st, exp = _merge_fixture()
    out, _ = merge_and_devices(st.reshape(5, -1), devices=[0, 0, 0])
    np.testing.assert_array_equal(out.reshape(3, -1), exp)
    out, _ = merge_and_devices(st.reshape(5, -1), devices=[0] * 7)  # workers with no state
    np.testing.assert_array_equal(out.reshape(3, -1), exp)
    odd = _states(37, 1000, 5)  # not a multiple of 16 bytes
    out, _ = merge_and_devices(odd, devices=[0, 0])
    np.testing.assert_array_equal(out, np.bitwise_and.reduce(odd, axis=0))
    out, _ = merge_and_devices(np.zeros((0, 96), np.uint8), devices=[0, 0])
    assert (out == 0xFF).all()


@pytest.mark.gpu
def test_merge_devices_errors(gpu):
    st = _states(10, 256, 3)
    with pytest.raises(RuntimeError, match="distinct"):
        merge_and_devices(st, devices=[0, 0], exchange=EXCHANGE_RCCL)
    with pytest.raises(RuntimeError, match="out of range"):
        merge_and_devices(st, devices=[0, 999])


def _rccl_mapped():
    with open("/proc/self/maps") as f:
        return any("librccl" in line for line in f)


@pytest.mark.gpu
def test_merge_devices_rccl_one_rank(gpu):
    """The RCCL exchange itself (dlopen'd librccl, ncclCommInitAll, grouped ncclAllGather, local
    AND, streams drained before the comms are destroyed) on one distinct device: the reference's
    golden merge (afl_merge over tests/golden/merge.npz) and a random fold."""
    from tests.test_golden import _merge_fixture

    st, exp = _merge_fixture()
    out, used = merge_and_devices(st.reshape(5, -1), devices=[0], exchange=EXCHANGE_RCCL)
    assert used == EXCHANGE_RCCL
    np.testing.assert_array_equal(out.reshape(3, -1), exp)
    big = _states(3000, 3 * 65536, 21)
    out, used = merge_and_devices(big, devices=[0], exchange=EXCHANGE_RCCL)
    assert used == EXCHANGE_RCCL
    np.testing.assert_array_equal(out, np.bitwise_and.reduce(big, axis=0))
    assert _rccl_mapped(), "librccl was not loaded"


@pytest.mark.gpu
def test_merge_devices_distinct_gpus(gpu):
    """Two or more distinct GPUs: AUTO takes RCCL (or falls back to copies if an RCCL step
    fails), both exchanges forced; every result is the AND.  Skipped on a one-GPU box."""
    import torch

    nd = torch.cuda.device_count()
    if nd < 2:
        pytest.skip("needs two or more GPUs")
    st = _states(4001, 3 * 8192, 33)
    exp = np.bitwise_and.reduce(st, axis=0)
    for ex in (None, EXCHANGE_COPY, EXCHANGE_RCCL):
        kw = {} if ex is None else {"exchange": ex}
        out, used = merge_and_devices(st, devices=list(range(nd)), **kw)
        if ex is not None:
            assert used == ex
        np.testing.assert_array_equal(out, exp)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["afl_gpu", "dynamorio_gpu"])
def test_merge_files_on_several_workers(gpu, name, tmp_path):
    """The merger's file loop through merge_files with merge_devices: files decoded concurrently
    by every worker's fill, the same maps as the one-GPU fold and as the AND."""
    n, m = 700, 8192
    keys = ("virgin_bits", "virgin_tmout", "virgin_crash") if name == "afl_gpu" else ("virgin_bits",)
    rng = np.random.default_rng(9)
    maps = {k: _states(n, m, int(rng.integers(1 << 30))) for k in keys}
    paths = []
    for i in range(n):
        pth = tmp_path / f"s{i}.json"
        pth.write_text(P.state_json({k: maps[k][i] for k in keys}, m))
        paths.append(str(pth))
    one = P.state_maps(P.Plugin.merge_files(name, f'{{"map_size": {m}}}', paths).get_state(), m)
    for devs in ("[0, 0]", "[0, 0, 0, 0]"):
        got = P.state_maps(P.Plugin.merge_files(
            name, f'{{"map_size": {m}, "merge_devices": {devs}}}', paths).get_state(), m)
        for k in keys:
            np.testing.assert_array_equal(got[k], np.bitwise_and.reduce(maps[k], axis=0))
            np.testing.assert_array_equal(got[k], one[k])
    with pytest.raises(RuntimeError, match="Could not read"):
        P.Plugin.merge_files(name, f'{{"map_size": {m}, "merge_devices": [0, 0]}}',
                             paths[:5] + [str(tmp_path / "nope.json")])


def test_merge_devices_option_is_validated():
    for bad in ('"some"', '[]', '["x"]', '[-1]', '{}'):
        with pytest.raises(RuntimeError, match="merge_devices"):
            P.Plugin.merge_files("afl_gpu", f'{{"map_size": 256, "merge_devices": {bad}}}',
                                 ["/nonexistent"])
