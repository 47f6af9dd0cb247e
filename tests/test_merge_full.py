"""BASELINE config 4 at full size: the merger's AND-fold (merger/merger.c:79-99 -> afl_merge
afl_instrumentation.c:123-140) of 100,000 states x 3 x 64 KiB = 19.7 GB, device-resident,
through kbz_merge_and_device, against a plain PyTorch AND-reduction of the same states.

The states are all-0xff maps with each bit cleared with probability 2^-17 (the AND of 17
random bytes marks the cleared bits), generated on the device in chunks: over 100,000 states
about half of the bits survive the fold, so the result is neither all-zero nor all-ones.
(SURVEY.md §8(d)'s merger generator clears 2 % of the bits per state, which folds to zero.)"""
import pytest

from killerbeez_amd.triage import merge_and

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


def _and_reduce(x):
    """AND of the rows of a uint8 [r, b] CUDA tensor by halving (plain torch ops)."""
    import torch

    while x.shape[0] > 1:
        h = x.shape[0] // 2
        y = torch.bitwise_and(x[:h], x[h:2 * h])
        x = torch.cat([y, x[2 * h:]]) if x.shape[0] % 2 else y
    return x[0]


def test_full_size_config4(gpu):
    import torch

    n, nbytes, chunk = 100_000, 3 * 65536, 2_000
    g = torch.Generator(device="cuda")
    g.manual_seed(0xC0F4)
    states = torch.empty((n, nbytes), dtype=torch.uint8, device="cuda")
    ref = torch.full((nbytes,), 0xFF, dtype=torch.uint8, device="cuda")
    for lo in range(0, n, chunk):
        c = states[lo:lo + chunk]
        clear = torch.randint(0, 256, c.shape, dtype=torch.uint8, device="cuda", generator=g)
        for _ in range(16):
            clear &= torch.randint(0, 256, c.shape, dtype=torch.uint8, device="cuda",
                                   generator=g)
        torch.bitwise_not(clear, out=c)
        ref &= _and_reduce(c)
        del clear
    got = merge_and(states)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)
    # AND-fold invariants: the result only clears bits, every state covers it, and it is
    # order-independent (the two halves folded separately give the same result)
    assert int((got & ~states[12345]).count_nonzero()) == 0
    halves = torch.bitwise_and(merge_and(states[: n // 2]), merge_and(states[n // 2:]))
    torch.cuda.synchronize()
    assert torch.equal(halves, got)
    # P(a bit survives) = (1 - 2^-17)^100000 = 0.47
    import numpy as np

    ones = int(np.unpackbits(got.cpu().numpy()).sum())
    assert 0.40 < ones / (8 * nbytes) < 0.55
