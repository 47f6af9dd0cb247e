"""The instrumentation_t-layout plugins of libkbz_plugin.so (include/kbz_plugin.h).

CPU part: the factory fills the reference's vtable order (instrumentation/instrumentation.h:
40-62) plus the appended members, options/state JSON round-trips without touching a GPU, and
every call that needs the GPU fails loudly instead of falling back to a CPU path.

GPU part (-m gpu): the plugins driven the way fuzzer/main.c:370-418 drives a plugin (one exec
at a time, is_new_path after each) and in deferred/batched form, bit-exact against the oracle's
sequential per-exec loop; state dump/load and the merger fold against the oracle.
"""
import ctypes as C
import json
import os

import numpy as np
import pytest

import oracle
from killerbeez_amd import plugin as P
from killerbeez_amd import synth

M = 4096


def _fn_addr(name):
    return C.cast(getattr(P.lib(), name), C.c_void_p).value


# ---- CPU ----------------------------------------------------------------------------------------

def test_factory_vtable_order():
    L = P.lib()
    assert C.sizeof(P.VTable) == 14 * 8
    for name in P.PLUGINS:
        vt = L.kbz_instrumentation_factory(name.encode())
        assert vt
        v = vt.contents
        for member in ("create", "cleanup", "merge", "get_state", "free_state", "set_state",
                       "enable", "is_new_path", "get_fuzz_result", "is_process_done",
                       "triage_batch", "merge_many"):
            assert getattr(v, member) == _fn_addr(f"kbz_{name}_{member}"), (name, member)
        if name == "afl_gpu":  # the afl plugin binds neither (instrumentation_factory.c:72-84)
            assert v.get_module_info is None and v.get_edges is None
        else:                  # dynamorio binds both (instrumentation_factory.c:53-54)
            assert v.get_module_info == _fn_addr("kbz_dynamorio_gpu_get_module_info")
            assert v.get_edges == _fn_addr("kbz_dynamorio_gpu_get_edges")
        C.CDLL(None).free(vt)
    assert not L.kbz_instrumentation_factory(b"afl")


@pytest.mark.parametrize("name", P.PLUGINS)
def test_state_roundtrip_without_gpu(name):
    rng = np.random.default_rng(3)
    maps = {"virgin_bits": rng.integers(0, 256, M).astype(np.uint8)}
    if name == "afl_gpu":
        maps["virgin_tmout"] = rng.integers(0, 256, M).astype(np.uint8)
        maps["virgin_crash"] = rng.integers(0, 256, M).astype(np.uint8)
    else:
        maps["last_shm_hash"] = 0xDEADBEEF
    st = P.state_json(maps, M)
    p = P.Plugin(name, f'{{"map_size": {M}, "max_batch": 8}}', st)
    back = P.state_maps(p.get_state(), M)
    for k, v in maps.items():
        if k == "last_shm_hash":
            assert back[k] == v
        else:
            np.testing.assert_array_equal(back[k], v)
    # fresh state: all-0xff maps (setup_shm afl_instrumentation.c:555-559)
    q = P.Plugin(name, f'{{"map_size": {M}}}')
    assert (P.state_maps(q.get_state(), M)["virgin_bits"] == 0xFF).all()
    # reference error values
    assert q.is_new_path() == -1            # before any exec
    assert q.get_fuzz_result() == P.FUZZ_ERROR
    assert q.enable() == -1 and "process control" in P.last_error()
    assert q.is_process_done() == -1
    assert q.set_state('{"map_size": 8192}') != 0
    assert q.set_state('{"virgin_bits": "zz"}') != 0


def test_dynamorio_state_keeps_last_process_status():
    """dynamorio_set_state restores last_process_status (:1325); get_state reports it until the
    next exec (a get -> set -> get round trip keeps it)."""
    opts = f'{{"map_size": {M}}}'
    st = P.state_json({"virgin_bits": np.full(M, 0xFF, np.uint8), "last_shm_hash": 7,
                       "last_path_was_new": 1, "last_process_status": P.FUZZ_CRASH}, M)
    p = P.Plugin("dynamorio_gpu", opts, st)
    back = P.state_maps(p.get_state(), M)
    assert back["last_process_status"] == P.FUZZ_CRASH and back["last_shm_hash"] == 7
    q = P.Plugin("dynamorio_gpu", opts, p.get_state())
    assert P.state_maps(q.get_state(), M)["last_process_status"] == P.FUZZ_CRASH
    assert q.get_fuzz_result() == P.FUZZ_ERROR  # no exec yet (the reference: enable not called)
    assert q.set_state(st.replace('"last_process_status": 2', '"last_process_status": -1')) != 0


def test_state_keys_are_top_level_only():
    """A key inside a nested object must not be taken for the top-level one: a per-module state's
    module objects repeat virgin_bits / last_shm_hash (dynamorio_get_state :1260-1275)."""
    v = np.full(M, 0xFF, np.uint8)
    v[3] = 0x12
    inner = bytes(np.zeros(M, np.uint8)).hex()
    st = ('{"map_size": %d, "decoy": {"virgin_bits": "%s", "last_shm_hash": 99}, '
          '"last_process_status": 0, "last_path_was_new": 0, "last_shm_hash": 5, '
          '"virgin_bits": "%s"}') % (M, inner, bytes(v).hex())
    p = P.Plugin("dynamorio_gpu", f'{{"map_size": {M}}}', st)
    back = P.state_maps(p.get_state(), M)
    np.testing.assert_array_equal(back["virgin_bits"], v)
    assert back["last_shm_hash"] == 5
    # a top-level key missing while a nested one exists: rejected, not read from the nest
    bad = '{"map_size": %d, "x": {"virgin_bits": "%s"}}' % (M, inner)
    assert p.set_state(bad) != 0
    # escapes in strings are decoded (module names), malformed text is an error
    opts = ('{"map_size": %d, "per_module_coverage": 1, "coverage_modules": ["a\\u00e9\\"b", '
            '"c"]}' % M)
    q = P.Plugin("dynamorio_gpu", opts)
    assert P.state_maps(q.get_state(), M)["modules"].keys() == {'a\u00e9"b', "c"}
    for broken in ('{"map_size": %d' % M, '{"map_size": -1}', '{"map_size": 4096,}',
                   '{"virgin_bits": "ff" "x"}', '[1, 2]', '{"a": [1, {"b": }]}', '',
                   '{"map_size": 99999999999999999999999}'):
        assert p.set_state(broken) != 0, broken


def test_bad_options_and_ignore_file(tmp_path):
    with pytest.raises(RuntimeError):
        P.Plugin("afl_gpu", '{"map_size": 1000}')
    bad = tmp_path / "ign.bin"
    bad.write_bytes(b"\0" * (M - 1))
    with pytest.raises(RuntimeError, match="Incorrect size"):
        P.Plugin("dynamorio_gpu", f'{{"map_size": {M}, "ignore_bytes_file": "{bad}"}}')
    good = tmp_path / "ign2.bin"
    good.write_bytes(b"\0" * M)
    P.Plugin("dynamorio_gpu", f'{{"map_size": {M}, "ignore_bytes_file": "{good}"}}').close()


def test_no_cpu_fallback():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    p = P.Plugin("afl_gpu", f'{{"map_size": {M}}}')
    t = np.zeros(M, np.uint8)
    t[5] = 1
    # the exec's trace goes straight into a pinned GPU ring slot: without a GPU, recording
    # fails and nothing computes on the CPU
    assert p.record(t, P.FUZZ_NONE) == -1
    assert "GPU" in P.last_error()
    assert p.is_new_path() == -1
    q = P.Plugin("afl_gpu", f'{{"map_size": {M}}}')
    with pytest.raises(RuntimeError, match="merge"):
        p.merge(q)


# ---- GPU ----------------------------------------------------------------------------------------

def _expected(mode, t, oc, virgin=None, ignore=None, last=0):
    return oracle.triage_batch(mode, t, oc, virgin=virgin, ignore=ignore, last_hash=last,
                               want=oracle.WANT_H32 | oracle.WANT_X64)


MODES = [("afl_gpu", oracle.MODE_AFL), ("dynamorio_gpu", oracle.MODE_DYNAMORIO)]


@pytest.mark.gpu
@pytest.mark.parametrize("name,mode", MODES)
def test_per_exec_like_fuzzer_main(gpu, name, mode):
    """fuzzer/main.c:374-385: one exec, then is_new_path; repeated."""
    t, oc = synth.sparse_np(150, M, seed=21, hot_frac=0.05, outcome_p=(0.8, 0.1, 0.1))
    t[40] = t[39]
    oc[40] = oc[39]
    exp = _expected(mode, t, oc)
    p = P.Plugin(name, f'{{"map_size": {M}, "max_batch": 16}}')
    for j in range(t.shape[0]):
        ticket = p.record(t[j], int(oc[j]))
        assert ticket == j
        assert p.is_new_path() == int(exp["hnb"][j] != 0), j
        assert p.result(ticket) == exp["hnb"][j]
        assert p.get_fuzz_result() == oc[j]
    got = P.state_maps(p.get_state(), M)
    np.testing.assert_array_equal(got["virgin_bits"], exp["virgin"][0])
    if name == "afl_gpu":
        np.testing.assert_array_equal(got["virgin_tmout"], exp["virgin"][1])
        np.testing.assert_array_equal(got["virgin_crash"], exp["virgin"][2])
    else:
        assert got["last_shm_hash"] == exp["last_hash"]


@pytest.mark.gpu
@pytest.mark.parametrize("name,mode", MODES)
def test_deferred_and_batched(gpu, name, mode):
    t, oc = synth.sparse_np(300, M, seed=22, hot_frac=0.05, outcome_p=(0.8, 0.1, 0.1))
    exp = _expected(mode, t, oc)
    p = P.Plugin(name, f'{{"map_size": {M}, "max_batch": 512}}')
    tickets = [p.record(t[j], int(oc[j])) for j in range(100)]  # queued, not yet triaged
    got = [p.result(k) for k in tickets]                         # one GPU batch of 100
    np.testing.assert_array_equal(np.array(got, np.uint8), exp["hnb"][:100])
    r = p.triage_batch(t[100:], oc[100:])                        # appended batched member
    np.testing.assert_array_equal(r["hnb"], exp["hnb"][100:])
    np.testing.assert_array_equal(r["h32"], exp["h32"][100:])
    np.testing.assert_array_equal(r["x64"], exp["x64"][100:])
    np.testing.assert_array_equal(P.state_maps(p.get_state(), M)["virgin_bits"], exp["virgin"][0])


@pytest.mark.gpu
@pytest.mark.parametrize("name,mode", MODES)
def test_deferred_windows_with_early_copies(gpu, name, mode):
    """Windows of more than 128 recorded execs start copying every 64 execs while recording
    (kbz_ring_commit); windows of 200, 256 (one full max_batch: flushed by the next record) and
    130 execs, with repeats across the commit points, equal the sequential per-exec results."""
    n = 200 + 256 + 1 + 130
    t, oc = synth.sparse_np(n, M, seed=23, hot_frac=0.05, outcome_p=(0.8, 0.1, 0.1))
    t[128] = t[127]
    t[192:200] = t[191]
    t[200 + 64] = t[200 + 63]
    exp = _expected(mode, t, oc)
    p = P.Plugin(name, f'{{"map_size": {M}, "max_batch": 256}}')
    got, lo = [], 0
    for w in (200, 257, 130):
        tickets = [p.record(t[j], int(oc[j])) for j in range(lo, lo + w)]
        got += [p.result(k) for k in tickets]
        lo += w
    np.testing.assert_array_equal(np.array(got, np.uint8), exp["hnb"])
    got_maps = P.state_maps(p.get_state(), M)
    np.testing.assert_array_equal(got_maps["virgin_bits"], exp["virgin"][0])
    if name == "dynamorio_gpu":
        assert got_maps["last_shm_hash"] == exp["last_hash"]


@pytest.mark.gpu
@pytest.mark.parametrize("sub_k", [1, 4, 8])
def test_afl_sub_batched_windows(gpu, monkeypatch, sub_k):
    """afl_gpu with KBZ_PLUGIN_SUBBATCH: small windows go to the GPU in parts of sub_k execs
    while recording continues (alternating ring slots); windows of 1, 3, sub_k, sub_k + 1, 16,
    70 (sub-batches up to 64 rows, then one part) and 200 (early commits in its last part), plus
    a query of an older ticket of the window and of the window before, equal the per-exec
    results."""
    monkeypatch.setenv("KBZ_PLUGIN_SUBBATCH", str(sub_k))
    wins = [1, 3, sub_k, sub_k + 1, 16, 70, 200]
    n = sum(wins)
    t, oc = synth.sparse_np(n, M, seed=31 + sub_k, hot_frac=0.05, outcome_p=(0.8, 0.1, 0.1))
    exp = _expected(oracle.MODE_AFL, t, oc)
    p = P.Plugin("afl_gpu", f'{{"map_size": {M}, "max_batch": 256}}')
    got, lo = [], 0
    for w in wins:
        tickets = [p.record(t[j], int(oc[j])) for j in range(lo, lo + w)]
        assert tickets == list(range(lo, lo + w))
        got += [p.result(k) for k in tickets]
        assert p.result(tickets[0]) == exp["hnb"][lo]  # an older ticket of this window
        lo += w
    np.testing.assert_array_equal(np.array(got, np.uint8), exp["hnb"])
    maps = P.state_maps(p.get_state(), M)
    np.testing.assert_array_equal(maps["virgin_bits"], exp["virgin"][0])
    np.testing.assert_array_equal(maps["virgin_tmout"], exp["virgin"][1])
    np.testing.assert_array_equal(maps["virgin_crash"], exp["virgin"][2])


@pytest.mark.gpu
@pytest.mark.parametrize("name,mode", MODES)
def test_sharded_windows_and_batches(gpu, name, mode):
    """Option "devices" (here two workers on one GPU, "0,0") with shard_min 64: recorded windows
    of 100 and 256 execs and a triage_batch of 300 (chunks of max_batch 256 and 44) go through
    kbz_triage_batch_devices, a window of 30 and the batch's last 44 through the plugin's own
    context; repeats at the window and shard boundaries (the DynamoRIO last-hash skip across
    them).  Results and the final state equal the per-exec ones."""
    wins = [100, 30, 256]
    n = sum(wins) + 300
    t, oc = synth.sparse_np(n, M, seed=41, hot_frac=0.05, outcome_p=(0.8, 0.1, 0.1))
    for j in (100, 130, 130 + 128, 386, 386 + 150):  # window / shard starts repeat their predecessor
        t[j] = t[j - 1]
        oc[j] = oc[j - 1]
    exp = _expected(mode, t, oc)
    opts = json.dumps({"map_size": M, "max_batch": 256, "devices": "0,0", "shard_min": 64})
    p = P.Plugin(name, opts)
    got, lo = [], 0
    for w in wins:
        tickets = [p.record(t[j], int(oc[j])) for j in range(lo, lo + w)]
        got += [p.result(k) for k in tickets]
        assert p.is_new_path() == int(exp["hnb"][lo + w - 1] != 0)
        lo += w
    r = p.triage_batch(t[lo:], oc[lo:], hashes=False)
    np.testing.assert_array_equal(np.array(got, np.uint8), exp["hnb"][:lo])
    np.testing.assert_array_equal(r["hnb"], exp["hnb"][lo:])
    maps = P.state_maps(p.get_state(), M)
    np.testing.assert_array_equal(maps["virgin_bits"], exp["virgin"][0])
    if name == "afl_gpu":
        np.testing.assert_array_equal(maps["virgin_tmout"], exp["virgin"][1])
        np.testing.assert_array_equal(maps["virgin_crash"], exp["virgin"][2])
    else:
        assert maps["last_shm_hash"] == exp["last_hash"]


def test_shard_options_are_checked():
    for bad in ('{"devices": 3}', '{"devices": "0,x"}', '{"devices": "-1"}', '{"shard_min": 0}'):
        with pytest.raises(RuntimeError):
            P.Plugin("afl_gpu", bad)


@pytest.mark.gpu
def test_dynamorio_ignore_file(gpu, tmp_path):
    rng = np.random.default_rng(4)
    ign = np.where(rng.random(M) < 0.4, 0, rng.integers(1, 256, M)).astype(np.uint8)
    f = tmp_path / "ignore.bin"
    f.write_bytes(ign.tobytes())
    t, oc = synth.sparse_np(120, M, seed=23, hot_frac=0.05)
    exp = _expected(oracle.MODE_DYNAMORIO, t, oc, ignore=ign)
    p = P.Plugin("dynamorio_gpu", f'{{"map_size": {M}, "ignore_bytes_file": "{f}"}}')
    r = p.triage_batch(t, oc)
    np.testing.assert_array_equal(r["hnb"], exp["hnb"])
    np.testing.assert_array_equal(r["h32"], exp["h32"])


@pytest.mark.gpu
@pytest.mark.parametrize("name,mode", MODES)
def test_state_load_continue_and_merge(gpu, name, mode):
    t, oc = synth.sparse_np(200, M, seed=24, hot_frac=0.05, outcome_p=(0.8, 0.1, 0.1))
    a = P.Plugin(name, f'{{"map_size": {M}}}')
    a.triage_batch(t[:100], oc[:100])
    # -isf/-isd style: dump, load into a new state, continue (fuzzer/main.c:300-322, :426-436)
    b = P.Plugin(name, f'{{"map_size": {M}}}', a.get_state())
    r = b.triage_batch(t[100:], oc[100:])
    if name == "afl_gpu":  # the loaded maps carry on (afl_instrumentation.c:553-559)
        np.testing.assert_array_equal(r["hnb"], _expected(mode, t, oc)["hnb"][100:])
    else:  # the first exec's enable resets virgin_bits, keeps the hash (test_dynamorio_resume)
        last = P.state_maps(a.get_state(), M)["last_shm_hash"]
        np.testing.assert_array_equal(r["hnb"], _expected(mode, t[100:], oc[100:], last=last)["hnb"])
    # merger: AND of the maps (afl_merge :123-140, dynamorio_merge :1180-1231)
    c = P.Plugin(name, f'{{"map_size": {M}}}')
    c.triage_batch(t[50:], oc[50:])
    m2 = a.merge(c)
    mm = P.Plugin.merge_many([a, b, c])
    va, vb, vc = (P.state_maps(x.get_state(), M) for x in (a, b, c))
    for k in va:
        if k == "last_shm_hash":
            continue
        np.testing.assert_array_equal(P.state_maps(m2.get_state(), M)[k], va[k] & vc[k])
        np.testing.assert_array_equal(P.state_maps(mm.get_state(), M)[k], va[k] & vb[k] & vc[k])
    if name == "dynamorio_gpu":
        assert P.state_maps(mm.get_state(), M)["last_shm_hash"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("name,mode", MODES)
def test_merge_files_like_the_merger(gpu, name, mode, tmp_path):
    """merger <plugin> out in_1 ... in_n (merger/merger.c:79-99): n state files folded in one
    GPU call (files decoded into pinned memory by worker threads), against the AND of the maps
    and the pairwise merge; more files than one staging slot holds; errors like the merger's."""
    rng = np.random.default_rng(7)
    n = 2100 if name == "afl_gpu" else 5000  # > 256 MiB / (3 x 16 KiB): several slots for AFL
    m = 16384
    keys = ("virgin_bits", "virgin_tmout", "virgin_crash") if name == "afl_gpu" else ("virgin_bits",)
    maps = {k: np.full((n, m), 0xFF, np.uint8) for k in keys}
    paths = []
    for i in range(n):
        st = {}
        for k in keys:
            clear = rng.random(m) < 0.002
            maps[k][i, clear] = rng.integers(0, 255, int(clear.sum()), dtype=np.uint8)
            st[k] = maps[k][i]
        if name == "dynamorio_gpu":
            st["last_shm_hash"] = int(rng.integers(1, 2**32))
        pth = tmp_path / f"state{i}.json"
        pth.write_text(P.state_json(st, m))
        paths.append(str(pth))
    opts = f'{{"map_size": {m}}}'
    merged = P.Plugin.merge_files(name, opts, paths)
    got = P.state_maps(merged.get_state(), m)
    for k in keys:
        np.testing.assert_array_equal(got[k], np.bitwise_and.reduce(maps[k], axis=0))
    if name == "dynamorio_gpu":
        assert got["last_shm_hash"] == 0
    # the pairwise fold of the merger gives the same maps
    a = P.Plugin(name, opts, open(paths[0]).read())
    for pth in paths[1:4]:
        a = a.merge(P.Plugin(name, opts, open(pth).read()))
    small = P.state_maps(P.Plugin.merge_files(name, opts, paths[:4]).get_state(), m)
    for k in keys:
        np.testing.assert_array_equal(small[k], P.state_maps(a.get_state(), m)[k])
    # errors: a missing file, a file with the wrong map size, nothing to merge
    with pytest.raises(RuntimeError, match="Could not read"):
        P.Plugin.merge_files(name, opts, paths[:3] + [str(tmp_path / "nope.json")])
    with pytest.raises(RuntimeError, match="map_size"):
        P.Plugin.merge_files(name, '{"map_size": 8192}', paths[:2])
    with pytest.raises(RuntimeError, match="nothing to merge"):
        P.Plugin.merge_files(name, opts, [])


@pytest.mark.gpu
def test_merge_files_per_module(gpu, tmp_path):
    """per_module_coverage states: modules matched by name in every file, module-wise AND."""
    m, names = 4096, ["a.dll", "b.exe", "c.so"]
    rng = np.random.default_rng(3)
    opts = f'{{"map_size": {m}, "per_module_coverage": 1, "coverage_modules": ["a.dll", "b.exe", "c.so"]}}'
    exp = {nm: np.full(m, 0xFF, np.uint8) for nm in names}
    paths = []
    for i in range(40):
        mods = {}
        for nm in reversed(names) if i % 2 else names:  # module order differs between files
            v = np.full(m, 0xFF, np.uint8)
            clear = rng.random(m) < 0.01
            v[clear] = rng.integers(0, 255, int(clear.sum()), dtype=np.uint8)
            exp[nm] &= v
            mods[nm] = {"virgin_bits": v, "last_shm_hash": i, "last_path_was_new": 0}
        pth = tmp_path / f"s{i}.json"
        pth.write_text(P.state_json({"modules": mods}, m))
        paths.append(str(pth))
    got = P.state_maps(P.Plugin.merge_files("dynamorio_gpu", opts, paths).get_state(), m)
    for nm in names:
        np.testing.assert_array_equal(got["modules"][nm]["virgin_bits"], exp[nm])
        assert got["modules"][nm]["last_shm_hash"] == 0
    bad = tmp_path / "bad.json"
    bad.write_text(P.state_json({"modules": {"a.dll": {"virgin_bits": exp["a.dll"]}}}, m))
    with pytest.raises(RuntimeError, match="lacks coverage module"):
        P.Plugin.merge_files("dynamorio_gpu", opts, paths[:2] + [str(bad)])


@pytest.mark.gpu
@pytest.mark.parametrize("name,mode", MODES)
def test_config1_real_traces_per_exec(gpu, name, mode):
    """BASELINE config 1 through the plugin as fuzzer/main.c:374-385 drives it (one exec, then
    is_new_path): the real afl-gcc traces of corpus/afl_test (tests/golden/config1.npz), whose
    expected results come from the reference's own code; "ABC@" reaches the crash."""
    f = np.load(os.path.join(os.path.dirname(__file__), "golden", "config1.npz"))
    key = "afl" if name == "afl_gpu" else "dynamorio"
    for tag in ("abc", "aaaa"):
        n = int(f[f"{tag}_n"])
        t = np.zeros((n, 65536), np.uint8)
        t[f[f"{tag}_tj"], f[f"{tag}_ti"]] = f[f"{tag}_tv"]
        oc = f[f"{tag}_outcome"]
        exp = f[f"{tag}_{key}_hnb"]
        p = P.Plugin(name, '{"map_size": 65536, "max_batch": 64}')
        for j in range(min(n, 300)):
            assert p.record(t[j], int(oc[j])) == j
            assert p.is_new_path() == int(exp[j] != 0), (tag, j)
            assert p.get_fuzz_result() == oc[j]
        p.close()


@pytest.mark.gpu
@pytest.mark.parametrize("per_module", [False, True])
def test_dynamorio_resume(gpu, per_module):
    """A resumed DynamoRIO campaign (fuzzer -isf: create(options, state), then execs).  The
    reference's first dynamorio_enable calls setup_shm_and_pick_fuzzer_id(state, 1)
    (dynamorio_instrumentation.c:1380-1382), which resets virgin_bits to 0xff (:496-497; every
    module's map with per_module_coverage, :458-459, :474-475) and keeps last_shm_hash.  So the
    per-exec results equal the oracle run from all-0xff maps with the restored hash; a set_state
    after an exec keeps the loaded maps; create + merge with no exec keeps them too."""
    import json

    n = 90
    mods = MODS if per_module else ["x"]
    k = len(mods)
    parts = [synth.sparse_np(2 * n, M, seed=80 + i, hot_frac=0.05)[0] for i in range(k)]
    for part in parts:
        part[n] = part[n - 1]  # the first resumed exec repeats the saved campaign's last exec
        part[n + 5:n + 9] = part[n + 4]
    rows = np.concatenate(parts, axis=1)
    opts = (PM_OPTS % (M, json.dumps(MODS))) if per_module else f'{{"map_size": {M}, "max_batch": 16}}'
    a = P.Plugin("dynamorio_gpu", opts)
    a.triage_batch(rows[:n], hashes=False)
    st = a.get_state()
    saved = P.state_maps(st, M)
    lasts = ([saved["modules"][nm]["last_shm_hash"] for nm in mods] if per_module
             else [saved["last_shm_hash"]])
    maps = ([saved["modules"][nm]["virgin_bits"] for nm in mods] if per_module
            else [saved["virgin_bits"]])
    assert all((mp != 0xFF).any() for mp in maps)  # the saved maps are not fresh
    exp = [oracle.triage_batch(oracle.MODE_DYNAMORIO, parts[i][n:], None, last_hash=lasts[i])
           for i in range(k)]
    # the saved maps would give other results: the reset is what makes these match
    old = [oracle.triage_batch(oracle.MODE_DYNAMORIO, parts[i][n:], None, last_hash=lasts[i],
                               virgin=np.stack([maps[i]] * 3)) for i in range(k)]
    want = np.any([e["hnb"] != 0 for e in exp], axis=0)
    assert not np.array_equal(want, np.any([e["hnb"] != 0 for e in old], axis=0))
    # create(options, state) then execs one at a time (fuzzer/main.c:374-385)
    b = P.Plugin("dynamorio_gpu", opts, st)
    for j in range(n):
        assert b.record(rows[n + j], P.FUZZ_NONE) == j
        assert b.is_new_path() == int(want[j]), j
    got = P.state_maps(b.get_state(), M)
    for i, nm in enumerate(mods):
        g = got["modules"][nm] if per_module else got
        np.testing.assert_array_equal(g["virgin_bits"], exp[i]["virgin"][0])
        assert g["last_shm_hash"] == exp[i]["last_hash"]
    # set_state after the first exec: the loaded maps are kept (fuzzer_id is set by then)
    b.set_state(st)
    r = b.triage_batch(rows[n:], hashes=False)
    np.testing.assert_array_equal(r["hnb"] != 0, np.any([e["hnb"] != 0 for e in old], axis=0))
    # the batched member resets too, on its first exec
    c = P.Plugin("dynamorio_gpu", opts, st)
    np.testing.assert_array_equal(c.triage_batch(rows[n:], hashes=False)["hnb"] != 0, want)
    # no exec, no enable: a loaded state merges with its maps
    d = P.Plugin("dynamorio_gpu", opts, st)
    m = d.merge(P.Plugin("dynamorio_gpu", opts))
    got = P.state_maps(m.get_state(), M)
    for i, nm in enumerate(mods):
        np.testing.assert_array_equal((got["modules"][nm] if per_module else got)["virgin_bits"],
                                      maps[i])


@pytest.mark.gpu
def test_afl_resume_keeps_loaded_maps(gpu):
    """afl_gpu: a loaded state's three maps carry on into the next execs
    (afl_instrumentation.c:553-559 fills only the maps it allocates)."""
    t, oc = synth.sparse_np(160, M, seed=81, hot_frac=0.05, outcome_p=(0.8, 0.1, 0.1))
    a = P.Plugin("afl_gpu", f'{{"map_size": {M}, "max_batch": 16}}')
    a.triage_batch(t[:80], oc[:80])
    b = P.Plugin("afl_gpu", f'{{"map_size": {M}, "max_batch": 16}}', a.get_state())
    exp = _expected(oracle.MODE_AFL, t, oc)
    for j in range(80, 160):
        b.record(t[j], int(oc[j]))
        assert b.is_new_path() == int(exp["hnb"][j] != 0), j


# ---- dynamorio_gpu per_module_coverage (dynamorio_instrumentation.c:1048-1063, :1477-1493) ----

MODS = ["target.exe", "lib_a.dll", "lib b.dll"]
PM_OPTS = '{"map_size": %d, "max_batch": 16, "per_module_coverage": 1, "coverage_modules": %s}'


def test_per_module_state_roundtrip_without_gpu():
    import json

    rng = np.random.default_rng(1239)
    mods = {name: {"virgin_bits": rng.integers(0, 256, M).astype(np.uint8),
                   "last_shm_hash": int(rng.integers(0, 2**32)), "last_path_was_new": i % 2}
            for i, name in enumerate(MODS)}
    opts = PM_OPTS % (M, json.dumps(MODS))
    st = P.state_json({"last_process_status": 0, "modules": dict(reversed(list(mods.items())))}, M)
    p = P.Plugin("dynamorio_gpu", opts, st)  # modules are matched by name, in any order
    back = P.state_maps(p.get_state(), M)
    assert list(back["modules"]) == MODS
    for name, m in mods.items():
        np.testing.assert_array_equal(back["modules"][name]["virgin_bits"], m["virgin_bits"])
        assert back["modules"][name]["last_shm_hash"] == m["last_shm_hash"]
        assert back["modules"][name]["last_path_was_new"] == m["last_path_was_new"]
    bad = P.state_json({"modules": {"other.dll": mods[MODS[0]]}}, M)
    assert p.set_state(bad) != 0 and "not a coverage module" in P.last_error()
    with pytest.raises(RuntimeError, match="coverage_modules"):
        P.Plugin("dynamorio_gpu", '{"map_size": %d, "per_module_coverage": 1}' % M)


@pytest.mark.gpu
def test_per_module_coverage_plugin(gpu, tmp_path):
    """record() takes the modules' maps back to back; is_new_path = any module new; each module
    keeps its own virgin map / ignore bytes (ignore_bytes_dir/<name>.dat) / last hash; state
    dump -> load -> continue; merge ANDs module by module (matched by name)."""
    import json

    rng = np.random.default_rng(1477)
    ign = np.where(rng.random(M) < 0.2, 0, 0xFF).astype(np.uint8)
    (tmp_path / f"{MODS[1]}.dat").write_bytes(ign.tobytes())
    opts = json.loads(PM_OPTS % (M, json.dumps(MODS)))
    opts["ignore_bytes_dir"] = str(tmp_path)
    opts = json.dumps(opts)
    k, n = len(MODS), 120
    parts = [synth.sparse_np(2 * n, M, seed=60 + i, hot_frac=0.05)[0] for i in range(k)]
    for part in parts:
        part[30:40] = part[29]
    rows = np.concatenate(parts, axis=1)
    igs = [None, ign, None]
    p = P.Plugin("dynamorio_gpu", opts)
    exp = [oracle.triage_batch(oracle.MODE_DYNAMORIO, parts[i][:n], None, ignore=igs[i])
           for i in range(k)]
    for j in range(n):
        assert p.record(rows[j], P.FUZZ_NONE) == j
        assert p.is_new_path() == int(any(e["hnb"][j] != 0 for e in exp)), j
    st = p.get_state()
    got = P.state_maps(st, M)["modules"]
    for i, name in enumerate(MODS):
        np.testing.assert_array_equal(got[name]["virgin_bits"], exp[i]["virgin"][0])
        assert got[name]["last_shm_hash"] == exp[i]["last_hash"]
        assert got[name]["last_path_was_new"] == int(exp[i]["hnb"][n - 1] != 0)
    # dump -> load into a new state -> the next execs continue from it: every module's map is
    # reset by the first exec's enable (dynamorio_instrumentation.c:458-459, :474-475), its last
    # hash is kept
    q = P.Plugin("dynamorio_gpu", opts, st)
    exp2 = [oracle.triage_batch(oracle.MODE_DYNAMORIO, parts[i][n:], None, ignore=igs[i],
                                last_hash=exp[i]["last_hash"])
            for i in range(k)]
    res = q.triage_batch(rows[n:], hashes=False)
    np.testing.assert_array_equal(res["hnb"], np.any([e["hnb"] != 0 for e in exp2], axis=0))
    # merge: module-wise AND
    m = p.merge(q)
    got = P.state_maps(m.get_state(), M)["modules"]
    for i, name in enumerate(MODS):
        np.testing.assert_array_equal(got[name]["virgin_bits"],
                                      exp[i]["virgin"][0] & exp2[i]["virgin"][0])
        assert got[name]["last_shm_hash"] == 0


# ---- get_module_info / get_edges / dump_map_dir (dynamorio_instrumentation.c:1541-1606, :1453) --

@pytest.mark.gpu
def test_get_module_info_like_the_picker(gpu):
    """picker/main.c:182-225 drives the plugin: per input file and iteration, test_input (here:
    record the exec's module maps) then get_module_info(index) for index = 0, 1, ... until it
    fails, collecting each module's is_new and trace map.  The maps must be the classified maps
    has_new_coverage leaves in trace_bits (:1434, :1565), is_new the module's has_new_coverage
    result for that exec; the collected maps then feed the picker's diff on the GPU
    (kbz_picker_ignore_device), checked against the restated picker loop."""
    import json

    import torch

    from killerbeez_amd.triage import picker_ignore

    files, iters, k = 3, 5, len(MODS)
    rng = np.random.default_rng(187)
    p = P.Plugin("dynamorio_gpu", PM_OPTS % (M, json.dumps(MODS)))
    assert p.get_module_info(0)[0] == -1          # no exec yet (enable_called)
    base = [[synth.sparse_np(1, M, seed=100 * f + i, hot_frac=0.05)[0][0] for i in range(k)]
            for f in range(files)]
    collected = np.zeros((k, files, iters, M), np.uint8)
    is_new = np.zeros((k, files * iters), np.int64)
    rows = []
    for f in range(files):
        for it in range(iters):
            maps = [b.copy() for b in base[f]]
            if it % 2:                              # module 1 is noisy on odd iterations
                maps[1][rng.choice(M, 3, replace=False)] = rng.integers(1, 256, 3)
            row = np.concatenate(maps)
            rows.append(row)
            assert p.record(row, P.FUZZ_NONE) >= 0  # driver->test_input
            index = 0
            while True:
                rc, nw, name, info = p.get_module_info(index)
                if rc:
                    assert rc == 1
                    break
                assert name == MODS[index] and info.size == M
                collected[index, f, it] = info
                is_new[index, f * iters + it] = nw
                index += 1
            assert index == k
    raw = np.array(rows)
    for i in range(k):
        part = raw[:, i * M:(i + 1) * M]
        exp = oracle.triage_batch(oracle.MODE_DYNAMORIO, part, None)
        np.testing.assert_array_equal(collected[i].reshape(-1, M), oracle.transform(part, 1))
        np.testing.assert_array_equal(is_new[i], (exp["hnb"] != 0).astype(np.int64))
        g_ign, g_pc, g_tot = picker_ignore(torch.from_numpy(collected[i]).cuda())
        torch.cuda.synchronize()
        ign, pc, tot = oracle.picker_ignore(collected[i])
        np.testing.assert_array_equal(g_ign.cpu().numpy(), ign)
        np.testing.assert_array_equal(g_pc.cpu().numpy().view(np.uint32), pc)
        assert int(g_tot.item()) == tot
        assert (tot > 0) == (i == 1)                # only the noisy module has ignore bytes
    assert p.get_edges(0) is None                   # no edge lists without the edges option
    # without per_module_coverage the coverage modules are named, without maps (as the reference)
    q = P.Plugin("dynamorio_gpu", '{"map_size": %d, "coverage_modules": ["t.exe"]}' % M)
    q.record(raw[0, :M], P.FUZZ_NONE)
    assert q.get_module_info(0) == (0, 0, "t.exe", None)
    assert q.get_module_info(1)[0] == 1


def _golden_config1(tag):
    f = np.load(os.path.join(os.path.dirname(__file__), "golden", "config1.npz"))
    n = int(f[f"{tag}_n"])
    t = np.zeros((n, 65536), np.uint8)
    t[f[f"{tag}_tj"], f[f"{tag}_ti"]] = f[f"{tag}_tv"]
    return t, f[f"{tag}_outcome"], f[f"{tag}_dynamorio_h32"]


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["record", "triage_batch"])
def test_dump_map_dir_config1(gpu, tmp_path, path):
    """dump_map_dir (dynamorio_instrumentation.c:1453-1458) on BASELINE config 1's real traces:
    every exec whose hash32 differs from the previous exec's writes its classified map to
    <dir>/<%08x hash>.  File names come from the reference build's own hashes (config1.npz),
    contents from the restated classify_counts."""
    import json

    t, oc, ref_h32 = _golden_config1("aaaa")
    t, oc, ref_h32 = t[:300], oc[:300], ref_h32[:300]
    d = tmp_path / "maps"
    d.mkdir()
    p = P.Plugin("dynamorio_gpu", json.dumps({"map_size": 65536, "max_batch": 64,
                                              "dump_map_dir": str(d)}))
    if path == "record":
        for j in range(t.shape[0]):
            p.record(t[j], int(oc[j]))
            if j % 37 == 0:
                assert p.is_new_path() >= 0         # flush windows of varying size
        assert p.flush() == 0
    else:
        p.triage_batch(t, oc, hashes=False)
    want, prev = {}, 0
    classified = oracle.transform(t, 1)
    for j, h in enumerate(ref_h32.tolist()):
        if h != prev:
            want[f"{h:08x}"] = classified[j]
        prev = h
    got = {x.name: np.frombuffer(x.read_bytes(), np.uint8) for x in d.iterdir()}
    assert set(got) == set(want) and len(want) > 1
    for name, m in want.items():
        np.testing.assert_array_equal(got[name], m)
