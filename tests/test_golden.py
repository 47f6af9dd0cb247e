"""Known-answer tests against tests/golden/*.npz (expected values produced by the reference's
own compiled code, see tests/golden/make_golden.py).

CPU tests pin the clean-room oracle to the fixtures; the gpu tests run the same vectors
through libkbz_hip.so's C ABI.
"""
import os

import numpy as np
import pytest

import oracle

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MODES = (("afl", oracle.MODE_AFL), ("dynamorio", oracle.MODE_DYNAMORIO),
         ("afl_classify", oracle.MODE_AFL_CLASSIFY))


def load(name):
    return np.load(os.path.join(G, name), allow_pickle=False)


def dense(n, m, j, i, v):
    t = np.zeros((n, m), np.uint8)
    t[j, i] = v
    return t


def virgin(m, vmap, vidx, vval):
    V = np.full((3, m), 0xFF, np.uint8)
    V[vmap, vidx] = vval
    return V


def test_tables(oracle_lib):
    f = load("tables.npz")
    np.testing.assert_array_equal(oracle.count_class_table(), f["count_class"])
    L = oracle.lib()
    for c in range(256):
        t = np.full(8, c, np.uint8)
        L.kbzo_simplify_trace(t.ctypes.data_as(oracle.C.c_void_p), 8)
        assert t[0] == f["simplify"][c]


def test_hashes(oracle_lib):
    f = load("hashes.npz")
    off = 0
    for k, n in enumerate(f["lens"]):
        b = f["bufs"][off:off + n]
        g = f["ignore"][off:off + n]
        off += n
        assert oracle.hash32(b) == f["hash32"][k]
        L = oracle.lib()
        hi = L.kbzo_hash32_with_ignore(b.ctypes.data_as(oracle.C.c_void_p),
                                       g.ctypes.data_as(oracle.C.c_void_p), int(n),
                                       oracle.HASH_CONST)
        assert hi == f["hash32_ignore"][k]
    for k, n in enumerate(f["xxh_lens"]):
        assert oracle.xxh64(f["xxh_buf"][:n], 0) == f["xxh64"][k]
        assert oracle.xxh64(f["xxh_buf"][:n], 0x9E3779B97F4A7C15) == f["xxh64_seeded"][k]


@pytest.mark.parametrize("name,mode", MODES)
def test_triage_oracle(oracle_lib, name, mode):
    f = load("triage.npz")
    m = int(f["map_size"])
    t = dense(int(f["n"]), m, f["tj"], f["ti"], f["tv"])
    r = oracle.triage_batch(mode, t, f["outcome"], want=oracle.WANT_H32 | oracle.WANT_X64)
    np.testing.assert_array_equal(r["hnb"], f[f"{name}_hnb"])
    np.testing.assert_array_equal(r["h32"], f[f"{name}_h32"])
    np.testing.assert_array_equal(r["x64"], f[f"{name}_x64"])
    np.testing.assert_array_equal(r["virgin"], virgin(m, f[f"{name}_vmap"], f[f"{name}_vidx"],
                                                      f[f"{name}_vval"]))
    if mode == oracle.MODE_DYNAMORIO:
        assert r["last_hash"] == f["dynamorio_last"]


def test_triage_ignore_oracle(oracle_lib):
    f = load("triage.npz")
    m = int(f["map_size"])
    t = dense(int(f["ign_n"]), m, f["ign_tj"], f["ign_ti"], f["ign_tv"])
    r = oracle.triage_batch(oracle.MODE_DYNAMORIO, t, None, ignore=f["ign_bytes"])
    np.testing.assert_array_equal(r["hnb"], f["ign_hnb"])
    np.testing.assert_array_equal(r["h32"], f["ign_h32"])
    np.testing.assert_array_equal(r["virgin"][0], virgin(m, f["ign_vmap"], f["ign_vidx"],
                                                         f["ign_vval"])[0])
    assert r["last_hash"] == f["ign_last"]


def _merge_fixture():
    f = load("merge.npz")
    st = np.full((5, 3, 65536), 0xFF, np.uint8)
    st[f["s_state"], f["s_map"], f["s_idx"]] = f["s_val"]
    exp = virgin(65536, f["m_map"], f["m_idx"], f["m_val"])
    return st, exp


def test_merge_oracle(oracle_lib):
    st, exp = _merge_fixture()
    np.testing.assert_array_equal(oracle.merge_many(st.reshape(5, -1)).reshape(3, -1), exp)


# ---- the gfx950 path on the same vectors -----------------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("pass1", ["narrow", "wide"])
@pytest.mark.parametrize("name,mode", MODES)
def test_triage_gpu(gpu, name, mode, pass1):
    import torch

    from killerbeez_amd.triage import WANT_H32, WANT_X64, TriageContext

    f = load("triage.npz")
    m = int(f["map_size"])
    t = dense(int(f["n"]), m, f["tj"], f["ti"], f["tv"])
    with TriageContext(m, mode, t.shape[0], pass1=pass1) as ctx:
        out = ctx.triage(torch.from_numpy(t).cuda(), torch.from_numpy(f["outcome"]).cuda(),
                         WANT_H32 | WANT_X64)
        torch.cuda.synchronize()
        ctx.sync()
        np.testing.assert_array_equal(out["hnb"].cpu().numpy(), f[f"{name}_hnb"])
        np.testing.assert_array_equal(out["h32"].cpu().numpy().view(np.uint32), f[f"{name}_h32"])
        np.testing.assert_array_equal(out["x64"].cpu().numpy().view(np.uint64), f[f"{name}_x64"])
        np.testing.assert_array_equal(ctx.get_virgin(), virgin(m, f[f"{name}_vmap"],
                                                               f[f"{name}_vidx"], f[f"{name}_vval"]))
        if mode == oracle.MODE_DYNAMORIO:
            assert ctx.last_hash == f["dynamorio_last"]


@pytest.mark.gpu
@pytest.mark.parametrize("pass1", ["narrow", "wide"])
def test_triage_ignore_gpu(gpu, pass1):
    import torch

    from killerbeez_amd.triage import WANT_H32, TriageContext

    f = load("triage.npz")
    m = int(f["map_size"])
    t = dense(int(f["ign_n"]), m, f["ign_tj"], f["ign_ti"], f["ign_tv"])
    with TriageContext(m, oracle.MODE_DYNAMORIO, t.shape[0], pass1=pass1) as ctx:
        ctx.set_ignore(f["ign_bytes"])
        out = ctx.triage(torch.from_numpy(t).cuda(), None, WANT_H32)
        torch.cuda.synchronize()
        ctx.sync()
        np.testing.assert_array_equal(out["hnb"].cpu().numpy(), f["ign_hnb"])
        np.testing.assert_array_equal(out["h32"].cpu().numpy().view(np.uint32), f["ign_h32"])
        np.testing.assert_array_equal(ctx.get_virgin()[0], virgin(m, f["ign_vmap"],
                                                                  f["ign_vidx"], f["ign_vval"])[0])
        assert ctx.last_hash == f["ign_last"]


@pytest.mark.gpu
def test_merge_gpu(gpu):
    import torch

    from killerbeez_amd.triage import merge_and

    st, exp = _merge_fixture()
    got = merge_and(torch.from_numpy(st.reshape(5, -1)).cuda())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(got.cpu().numpy().reshape(3, -1), exp)


# ---- picker ignore-bytes diff (picker/main.c:240-262) ----------------------------------------

def _picker_fixture():
    f = load("picker.npz")
    F, I, S = (int(x) for x in f["shape"])
    runs = np.zeros((F, I, S), np.uint8)
    runs[f["r_file"], f["r_iter"], f["r_idx"]] = f["r_val"]
    ign = np.full(S, 0xFF, np.uint8)
    ign[f["ign_zero"]] = 0
    assert list(f["ign_other"]) == [0xFF]
    return runs, ign, f["pair_counts"], int(f["total"])


def test_picker_oracle(oracle_lib):
    runs, ign, pc, tot = _picker_fixture()
    g_ign, g_pc, g_tot = oracle.picker_ignore(runs)
    np.testing.assert_array_equal(g_ign, ign)
    np.testing.assert_array_equal(g_pc, pc)
    assert g_tot == tot


@pytest.mark.gpu
def test_picker_gpu(gpu):
    import torch

    from killerbeez_amd.triage import picker_ignore

    runs, ign, pc, tot = _picker_fixture()
    g_ign, g_pc, g_tot = picker_ignore(torch.from_numpy(runs).cuda())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(g_ign.cpu().numpy(), ign)
    np.testing.assert_array_equal(g_pc.cpu().numpy().view(np.uint32), pc)
    assert int(g_tot.item()) == tot


# ---- BASELINE config 1: real afl-gcc traces of corpus/afl_test (tests/golden/make_config1.py) --

C1_SEQS = ("aaaa", "abc")
C1_MODES = (("afl", oracle.MODE_AFL), ("dynamorio", oracle.MODE_DYNAMORIO))


def c1_traces(f, tag):
    n = int(f[f"{tag}_n"])
    return dense(n, 65536, f[f"{tag}_tj"], f[f"{tag}_ti"], f[f"{tag}_tv"]), f[f"{tag}_outcome"]


def test_config1_fixture_sanity(oracle_lib):
    """The captured runs behave as the reference's smoke test expects (sanity, not parity: the
    bit_flip mutator is external): tests/smoke_test.sh:139-145 wants 2 new paths in 10 execs
    from "AAAA", :172-175 a crash from "ABC@"."""
    f = load("config1.npz")
    assert int(f["smoke_new_paths"]) == 2
    assert (f["abc_outcome"] == oracle.FUZZ_CRASH).sum() >= 1
    assert (f["aaaa_outcome"] == oracle.FUZZ_NONE).all()


@pytest.mark.parametrize("tag", C1_SEQS)
@pytest.mark.parametrize("name,mode", C1_MODES)
def test_config1_oracle(oracle_lib, tag, name, mode):
    f = load("config1.npz")
    t, oc = c1_traces(f, tag)
    r = oracle.triage_batch(mode, t, oc, want=oracle.WANT_H32 | oracle.WANT_X64)
    np.testing.assert_array_equal(r["hnb"], f[f"{tag}_{name}_hnb"])
    np.testing.assert_array_equal(r["h32"], f[f"{tag}_{name}_h32"])
    np.testing.assert_array_equal(r["x64"], f[f"{tag}_{name}_x64"])
    np.testing.assert_array_equal(r["virgin"], virgin(65536, f[f"{tag}_{name}_vmap"],
                                                      f[f"{tag}_{name}_vidx"],
                                                      f[f"{tag}_{name}_vval"]))
    if mode == oracle.MODE_DYNAMORIO:
        assert r["last_hash"] == int(f[f"{tag}_{name}_last"])


@pytest.mark.gpu
@pytest.mark.parametrize("pass1", ["narrow", "wide"])
@pytest.mark.parametrize("split", [0, 7, 64])
@pytest.mark.parametrize("tag", C1_SEQS)
@pytest.mark.parametrize("name,mode", C1_MODES)
def test_config1_gpu(gpu, tag, name, mode, split, pass1):
    """The real traces through libkbz_hip.so: one batch (split 0) or consecutive batches of
    `split` execs with the state carried, against the reference's own per-exec results."""
    import torch

    from killerbeez_amd.triage import WANT_H32, WANT_X64, TriageContext

    f = load("config1.npz")
    t, oc = c1_traces(f, tag)
    n = t.shape[0]
    step = split or n
    hnb, h32, x64 = [], [], []
    with TriageContext(65536, mode, step, pass1=pass1) as ctx:
        for lo in range(0, n, step):
            out = ctx.triage(torch.from_numpy(t[lo:lo + step]).cuda(),
                             torch.from_numpy(oc[lo:lo + step]).cuda(), WANT_H32 | WANT_X64)
            torch.cuda.synchronize()
            ctx.sync()
            hnb.append(out["hnb"].cpu().numpy())
            h32.append(out["h32"].cpu().numpy().view(np.uint32))
            x64.append(out["x64"].cpu().numpy().view(np.uint64))
        np.testing.assert_array_equal(np.concatenate(hnb), f[f"{tag}_{name}_hnb"])
        np.testing.assert_array_equal(np.concatenate(h32), f[f"{tag}_{name}_h32"])
        np.testing.assert_array_equal(np.concatenate(x64), f[f"{tag}_{name}_x64"])
        np.testing.assert_array_equal(ctx.get_virgin(), virgin(65536, f[f"{tag}_{name}_vmap"],
                                                               f[f"{tag}_{name}_vidx"],
                                                               f[f"{tag}_{name}_vval"]))
        if mode == oracle.MODE_DYNAMORIO:
            assert ctx.last_hash == int(f[f"{tag}_{name}_last"])
