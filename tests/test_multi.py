"""The merger fold sharded over GPUs from C (kbz_merge_and_fill_devices, include/kbz_triage.h):
merger/merger.c:79-104 with the states split across workers, one per GPU (several may share a
GPU), exchanged by copies or RCCL and ANDed.  On a one-GPU box the workers share cuda:0 and the
copy path runs; the RCCL all-gather path needs distinct GPUs and is unmeasured here (it runs on a
multi-GPU node: its results are the same AND)."""
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
