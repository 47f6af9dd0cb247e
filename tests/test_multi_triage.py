"""Sharded triage over several GPUs of one node from C (kbz_mctx_*, kbz_triage_batch_devices;
include/kbz_triage.h): the protocol of killerbeez_amd.dist in one process,
workers exchanging link rows and OR aggregates by peer / device-local copies.  On a one-GPU box
the workers share cuda:0 (several contexts, device-local copies); the results must equal one
sequential pass of the CPU oracle over the whole batch, batch after batch (virgin maps and the
DynamoRIO last hash carried), with ragged and empty shards and repeats across shard boundaries."""
import numpy as np
import pytest

import oracle
from killerbeez_amd import synth
from killerbeez_amd.triage import WANT_H32, KbzError, MultiTriageContext

MODES = [0, 1, 2]


def _sharded_batches(mode, devices):
    m = 4096
    sizes = [700, 1001, 2, 0, 333]  # ragged shards; 2 and 0 traces leave workers empty
    v = np.full((3, m), 0xFF, np.uint8)
    last = 0
    with MultiTriageContext(m, mode, 512, devices=devices) as mc:
        assert mc.workers() == len(devices)
        for b, n in enumerate(sizes):
            t, oc = synth.sparse_np(n, m, seed=500 + 31 * b + mode, hot_frac=0.05)
            if n > 10:
                cut = n // len(devices)  # a repeat across the first shard boundary (DynamoRIO skip)
                t[cut] = t[cut - 1]
                t[n // 2 + 1] = t[n // 2]
                for j in (64, cut + 64, cut + 128):  # repeats at 64-row chunk starts inside a
                    if j < n:                        # shard: the pass-1 look-back's row compare
                        t[j] = t[j - 1]
            exp = oracle.triage_batch(mode, t, oc, virgin=v, last_hash=last, want=oracle.WANT_H32)
            got = mc.triage_host(t, oc, WANT_H32)
            np.testing.assert_array_equal(got["hnb"], exp["hnb"])
            if mode == 1 or n:
                np.testing.assert_array_equal(got["h32"], exp["h32"])
            np.testing.assert_array_equal(mc.get_virgin(), exp["virgin"])
            if mode == 1:
                assert mc.last_hash == exp["last_hash"]
            v, last = exp["virgin"], exp.get("last_hash", last)


@pytest.mark.gpu
@pytest.mark.parametrize("pass1", ["narrow", "wide"])
@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("workers", [2, 3])
def test_sharded_batches_from_c(gpu, mode, workers, pass1, monkeypatch):
    """Workers sharing cuda:0 (device-local copies).  Both pass-1 kernels: the shards here are a
    few chunks, which AUTO sends to the wide kernels; narrow forces k_pass1s, whose epilogue runs
    the skip rule (rows j >= 1 of a shard, with the look-back across its chunks)."""
    monkeypatch.setenv("KBZ_PASS1", pass1)
    _sharded_batches(mode, [0] * workers)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", MODES)
def test_sharded_batches_from_c_distinct_gpus(gpu, mode):
    """One worker per GPU (peer copies over xGMI); needs a multi-GPU node."""
    import torch

    if torch.cuda.device_count() < 2:
        pytest.skip("needs >= 2 GPUs")
    _sharded_batches(mode, list(range(min(torch.cuda.device_count(), 4))))


@pytest.mark.gpu
@pytest.mark.parametrize("mode", MODES)
def test_sharded_resident_batches_from_c(gpu, mode):
    """kbz_triage_batch_devices_resident: shards already on the devices (three workers sharing
    cuda:0, one of them empty), two batches in a row with repeats at the shard boundaries, equal
    to one sequential pass; then a host batch through the same context continues the state."""
    import torch

    m = 4096
    v = np.full((3, m), 0xFF, np.uint8)
    last = 0
    with MultiTriageContext(m, mode, 512, devices=[0, 0, 0]) as mc:
        assert mc.peer_pairs() == 0  # one distinct device: nothing to enable
        for b, counts in enumerate([(300, 0, 211), (64, 129, 1)]):
            n = sum(counts)
            t, oc = synth.sparse_np(n, m, seed=900 + 7 * b + mode, hot_frac=0.05)
            t[counts[0]] = t[counts[0] - 1] if counts[0] and n > counts[0] else t[counts[0]]
            exp = oracle.triage_batch(mode, t, oc, virgin=v, last_hash=last, want=oracle.WANT_H32)
            shards, ocs, lo = [], [], 0
            for c in counts:
                shards.append(torch.from_numpy(t[lo:lo + c].copy()).cuda())
                ocs.append(torch.from_numpy(oc[lo:lo + c].copy()).cuda())
                lo += c
            got = mc.triage_resident(shards, ocs, WANT_H32)
            hnb = np.concatenate([h.cpu().numpy() for h in got["hnb"]])
            np.testing.assert_array_equal(hnb, exp["hnb"])
            if mode == 1:
                h32 = np.concatenate([h.cpu().numpy().view(np.uint32) for h in got["h32"]])
                np.testing.assert_array_equal(h32, exp["h32"])
                assert mc.last_hash == exp["last_hash"]
            np.testing.assert_array_equal(mc.get_virgin(), exp["virgin"])
            v, last = exp["virgin"], exp.get("last_hash", last)
        t, oc = synth.sparse_np(400, m, seed=950 + mode, hot_frac=0.05)
        exp = oracle.triage_batch(mode, t, oc, virgin=v, last_hash=last, want=oracle.WANT_H32)
        np.testing.assert_array_equal(mc.triage_host(t, oc, WANT_H32)["hnb"], exp["hnb"])


@pytest.mark.gpu
def test_sharded_from_c_set_virgin_and_limits(gpu):
    m = 2048
    t, oc = synth.sparse_np(300, m, seed=9, hot_frac=0.05)
    with MultiTriageContext(m, 1, 100, devices=[0, 0]) as mc:
        pre = np.full((3, m), 0xFF, np.uint8)
        pre[0, : m // 2] = 0  # a preset map reaches every worker
        mc.set_virgin(pre)
        with pytest.raises(KbzError, match="max_batch"):
            mc.triage_host(t, oc)  # 150 traces per worker > 100
        got = mc.triage_host(t[:200], oc[:200])
        exp = oracle.triage_batch(1, t[:200], oc[:200], virgin=pre, want=oracle.WANT_H32)
        np.testing.assert_array_equal(got["hnb"], exp["hnb"])
        np.testing.assert_array_equal(mc.get_virgin(), exp["virgin"])
    with pytest.raises(KbzError, match="out of range"):
        MultiTriageContext(m, 1, 100, devices=[0, 999])


@pytest.mark.gpu
def test_sharded_from_c_ignore_bytes_and_restored_hash(gpu):
    """DynamoRIO ignore bytes on every worker and a restored last hash (the first row repeats the
    hash's trace: a skip), two batches, against the oracle with the same ignore bytes."""
    m = 4096
    rng = np.random.default_rng(77)
    ig = (rng.random(m) < 0.3).astype(np.uint8)
    t, oc = synth.sparse_np(600, m, seed=78, hot_frac=0.05)
    first = oracle.triage_batch(1, t[:1], oc[:1], want=oracle.WANT_H32)
    v = np.full((3, m), 0xFF, np.uint8)
    with MultiTriageContext(m, 1, 256, devices=[0, 0]) as mc:
        mc.set_ignore(ig)
        mc.last_hash = int(first["h32"][0])
        last = int(first["h32"][0])
        for b in range(2):
            part = t[300 * b:300 * (b + 1)].copy()
            if b == 0:
                part[0] = t[0]  # repeats the restored hash's trace
            exp = oracle.triage_batch(1, part, oc[300 * b:300 * (b + 1)], virgin=v, ignore=ig,
                                      last_hash=last, want=oracle.WANT_H32)
            got = mc.triage_host(part, oc[300 * b:300 * (b + 1)], WANT_H32)
            np.testing.assert_array_equal(got["hnb"], exp["hnb"])
            np.testing.assert_array_equal(got["h32"], exp["h32"])
            np.testing.assert_array_equal(mc.get_virgin(), exp["virgin"])
            assert mc.last_hash == exp["last_hash"]
            v, last = exp["virgin"], exp["last_hash"]
        assert exp is not None


def test_mctx_create_fails_loudly_without_a_device():
    """On a host with no GPU the multi-device context refuses to start (no CPU fallback)."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(KbzError, match="no device"):
        MultiTriageContext(1024, 0, 16, devices=[0])
