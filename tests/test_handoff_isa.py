"""The fused tail's in-launch hand-offs, checked on the compiled gfx950 ISA (CPU suite).

k_tail publishes its fix-path words with plain stores, then `s_barrier`, `buffer_wbl2 sc1`
(agent release), `s_waitcnt vmcnt(0)` and an `sc1` flag store; its readers poll `sc1`, acquire
(`buffer_inv sc1`) and wait before their barrier.  k_fin's copiers start from an agent-scope
ticket added after every wave drained its atomics and the workgroup barrier.  These are the valid
forms of MI355X_MICROARCH.md (inter-workgroup visibility); tools/handoff_isa_check.py asserts on
the ISA that every flag store and ticket is ordered after its payload.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_tail_handoffs_are_ordered(product_isa):
    import handoff_isa_check as H

    funcs = H.split_functions(product_isa.split("\n"))
    tail = [k for k in funcs if "k_tail" in k]
    fin = [k for k in funcs if "k_fin" in k]
    assert len(tail) == 1 and len(fin) == 1, sorted(funcs)[:10]
    issues, counts = H.check(funcs[tail[0]], tickets=False)
    assert not issues, issues[:5]
    # the fix path: two releases (walks done, column group fixed), three sc1 flag stores
    assert counts["wbl2"] == 2 and counts["flag_stores"] == 3 and counts["inv"] == 2, counts
    issues, counts = H.check(funcs[fin[0]], tickets=True)
    assert not issues, issues[:5]
    assert counts["tickets"] == 2 and counts["inv"] == 2, counts


def test_small_ticket_and_pass1_lookback(product_isa):
    """Every other kernel with an in-launch hand-off: k_small's last-workgroup ticket (drain,
    barrier, agent release waited for, returning atomic add; its sc1 dword stores re-arm words
    for the next launch) and k_pass1s's look-back in the fused skip rule (one 64-bit agent-scope
    word carrying tag and hash: a single sc1 dwordx2 store, polled by sc1 dwordx2 loads).  The
    staged kernels (k_skip, k_chain, k_total, k_scan, k_resolve, k_pack) hand nothing over
    inside a launch: their consumers are the next launches."""
    import handoff_isa_check as H

    funcs = H.split_functions(product_isa.split("\n"))
    small = [k for k in funcs if "k_small" in k]
    assert len(small) == 2, sorted(funcs)[:10]
    for k in small:
        issues, counts = H.check(funcs[k], tickets=True, flags=False)
        assert not issues, (k, issues[:5])
        assert counts["tickets"] == 1 and counts["wbl2"] == 1 and counts["inv"] == 1, counts
    p1s_dr = [k for k in funcs if "k_pass1s" in k and "k_pass1sILi1E" in k]
    assert len(p1s_dr) == 4, sorted(k for k in funcs if "k_pass1s" in k)
    for k in p1s_dr:
        pub, poll, other = H.lookback(funcs[k])
        assert len(pub) == 1 and len(poll) >= 1 and not other, (k, pub, poll, other)
    for k in funcs:  # the AFL-mode instantiations have no look-back at all
        if "k_pass1s" in k and k not in p1s_dr:
            assert H.lookback(funcs[k]) == ([], [], []), k
    staged = [k for k in funcs if any(f"{n}" in k for n in ("k_skip", "k_chain", "k_total",
                                                             "k_scan", "k_resolve", "k_pack"))]
    assert len(staged) >= 6
    for k in staged:
        b = funcs[k]
        assert not any(x.startswith("buffer_wbl2") or x.startswith("buffer_inv") for x in b), k


def test_checker_catches_unordered_handoffs():
    import handoff_isa_check as H

    store_then_flag = ["global_store_dwordx4 v0, v[2:5], s[0:1]",
                       "global_store_dword v0, v1, s[2:3] sc1"]
    assert H.check(store_then_flag)[0]
    release_not_waited = ["buffer_wbl2 sc1", "global_store_dword v0, v1, s[2:3] sc1"]
    assert H.check(release_not_waited)[0]
    ticket_no_barrier = ["global_atomic_umax v[2:3], v1, off", "s_waitcnt vmcnt(0)",
                         "global_atomic_add v2, v2, v3, s[10:11] sc0"]
    assert H.check(ticket_no_barrier)[0]
    acquire_not_waited = ["buffer_inv sc1", "s_barrier"]
    assert H.check(acquire_not_waited)[0]
    ok = ["global_store_dwordx4 v0, v[2:5], s[0:1]", "s_waitcnt vmcnt(0)", "s_barrier",
          "buffer_wbl2 sc1", "s_waitcnt vmcnt(0)", "global_store_dword v0, v1, s[2:3] sc1"]
    assert not H.check(ok)[0]
