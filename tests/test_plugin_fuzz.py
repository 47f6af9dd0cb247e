"""Property tests of the plugins' option / state JSON reader (killerbeez_amd/csrc/kbz_plugin.c).

The state and option strings arrive from files (the merger's state files, -isf / -isd in
fuzzer/main.c:300-322) and are parsed by hand-written C, so malformed, truncated and nested
input must be rejected cleanly -- never read past the string or crash -- and whatever is
accepted must be exactly the top-level values.  scripts/sanitize.sh runs this file against an
ASan + UBSan build of the plugin.  CPU only: no GPU call is reached (set_state / create /
get_state on a plugin that has not triaged anything).
"""
import json

import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from killerbeez_amd import plugin as P

M = 256  # smallest map: 3 x 512 hex digits per afl state
SETTINGS = settings(max_examples=150, deadline=None, derandomize=True,
                    suppress_health_check=[HealthCheck.too_slow])

json_leaf = st.one_of(st.none(), st.booleans(), st.integers(-2**70, 2**70),
                      st.floats(allow_nan=False, allow_infinity=False), st.text(max_size=12))
json_value = st.recursive(json_leaf, lambda kids: st.one_of(
    st.lists(kids, max_size=4), st.dictionaries(st.text(max_size=12), kids, max_size=4)),
    max_leaves=12)
KEYS = ["map_size", "virgin_bits", "virgin_tmout", "virgin_crash", "last_shm_hash",
        "last_path_was_new", "last_process_status", "modules", "name"]


def _maps(seed):
    rng = np.random.default_rng(seed)
    return {k: rng.integers(0, 256, M).astype(np.uint8)
            for k in ("virgin_bits", "virgin_tmout", "virgin_crash")}


def _afl_state(maps, extra=None):
    d = {"map_size": M}
    d.update({k: bytes(v).hex() for k, v in maps.items()})
    if extra:
        d.update(extra)
    return json.dumps(d)


@pytest.fixture(scope="module")
def afl():
    p = P.Plugin("afl_gpu", json.dumps({"map_size": M}))
    yield p
    p.close()


@SETTINGS
@given(text=st.one_of(st.text(max_size=200), st.binary(max_size=200).map(
    lambda b: b.decode("latin-1"))))
def test_arbitrary_text_is_rejected_cleanly(afl, text):
    """Random text as a state: rejected (or, if it happens to be a valid state, accepted) --
    the call returns either way; as options, create returns NULL or a plugin."""
    rc = afl.set_state(text.replace("\0", ""))
    assert rc in (0, 1)
    try:
        P.Plugin("dynamorio_gpu", text.replace("\0", "")).close()
    except RuntimeError:
        pass


@SETTINGS
@given(seed=st.integers(0, 2**32 - 1), cut=st.integers(0, 10**9))
def test_truncated_state_is_rejected(afl, seed, cut):
    s = _afl_state(_maps(seed))
    k = cut % len(s)
    assert afl.set_state(s[:k]) != 0


@SETTINGS
@given(seed=st.integers(0, 2**32 - 1),
       nested=st.dictionaries(st.sampled_from(KEYS), json_value, max_size=4),
       where=st.sampled_from(KEYS + ["zz"]))
def test_nested_keys_do_not_shadow_top_level(afl, seed, nested, where):
    """Objects nested anywhere (before or after the real keys) may repeat the state's key names;
    an accepted state holds exactly the top-level maps."""
    maps = _maps(seed)
    extra = {"a_nest": nested, where + "_x": [nested, {"k": nested}]}
    s = _afl_state(maps, extra)
    assert afl.set_state(s) == 0
    back = P.state_maps(afl.get_state(), M)
    for k, v in maps.items():
        np.testing.assert_array_equal(back[k], v)


@SETTINGS
@given(seed=st.integers(0, 2**32 - 1), key=st.sampled_from(
    ["virgin_bits", "virgin_tmout", "virgin_crash", "map_size"]), bad=json_value)
def test_wrong_typed_values_are_rejected(afl, seed, key, bad):
    maps = _maps(seed)
    d = json.loads(_afl_state(maps))
    d[key] = bad
    good = (key == "map_size" and isinstance(bad, int) and not isinstance(bad, bool)
            and bad == M)
    assert (afl.set_state(json.dumps(d)) == 0) == good


@SETTINGS
@given(names=st.lists(st.text(min_size=1, max_size=10).filter(lambda x: "\0" not in x),
                      min_size=1, max_size=4, unique=True))
def test_module_names_round_trip_with_escapes(names):
    """coverage_modules names with quotes, backslashes, control and non-ASCII characters are
    decoded (json_unquote) and written back escaped: get_state -> json.loads gives them back."""
    opts = json.dumps({"map_size": M, "per_module_coverage": 1, "coverage_modules": names})
    p = P.Plugin("dynamorio_gpu", opts)
    st_ = p.get_state()
    back = json.loads(st_)
    assert [m["name"] for m in back["modules"]] == names
    q = P.Plugin("dynamorio_gpu", opts, st_)
    assert json.loads(q.get_state())["modules"] == back["modules"]
