"""killerbeez_amd -- MI355X (gfx950) coverage-triage engine for Killerbeez.

The product is the C-ABI library ``libkbz_hip.so`` (include/kbz_triage.h) and the C plugin
``libkbz_plugin.so`` (include/kbz_plugin.h).  This package only holds their sources, the
build script, and thin host-side handles (ctypes) used by tests, bench and the multi-GPU
driver.  There is no CPU fallback: every entry point raises if the HIP library is missing.
"""
from .triage import (FUZZ_CRASH, FUZZ_HANG, FUZZ_NONE, MODE_AFL, MODE_AFL_CLASSIFY,  # noqa
                     MODE_DYNAMORIO, WANT_H32, WANT_X64, TriageContext, merge_and,
                     merge_and_host)

__all__ = ["TriageContext", "merge_and", "merge_and_host", "MODE_AFL", "MODE_DYNAMORIO",
           "MODE_AFL_CLASSIFY", "FUZZ_NONE", "FUZZ_HANG", "FUZZ_CRASH", "WANT_H32", "WANT_X64"]
