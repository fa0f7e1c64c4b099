import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_addoption(parser):
    parser.addoption("--force-record-lists", action="store_true", default=False,
                     help="every eligible TUMBLE handle keeps its state as record lists (FWA_CFG_RECORD_LISTS): runs "
                          "the parity suite over the sparse layout (tools/gpu_record_lists_suite.sh)")
    parser.addoption("--force-option", action="append", default=[], metavar="NAME=VALUE",
                     help="fwa_set_option applied to every handle of the session (engine.DEFAULT_OPTIONS), e.g. "
                          "window_passes=1 to run the parity suite over the combiner's window passes")


def _record_lists_eligible(c):
    """sp_eligible (flink_amd/csrc/sparse.inc): TUMBLE, no NULLs, UTC, no dynamic gap, lateness 0 for DataStream."""
    from flink_amd import _abi as A
    return (c.window_kind == 0 and c.nullable_cols == 0 and c.tz_n == 0 and not (c.flags & A.CFG_DYNAMIC_GAP)
            and (c.semantics == 1 or c.allowed_lateness_ms == 0))


def pytest_configure(config):
    if config.getoption("--force-record-lists"):
        from flink_amd import _abi as A
        make = A.make_config

        def make_forced(*a, **kw):
            c = make(*a, **kw)
            if _record_lists_eligible(c):
                c.flags |= A.CFG_RECORD_LISTS
            return c
        A.make_config = make_forced
    for opt in config.getoption("--force-option"):
        from flink_amd import engine
        name, _, value = opt.partition("=")
        engine.DEFAULT_OPTIONS[name] = int(value)
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine through the C-ABI)")
    config.addinivalue_line("markers", "slow: longer CPU test")
