"""Static check of bench.py and the host modules (no GPU): every name a function reads must be a
local, an enclosing-scope name, a module global or a builtin.  The GPU-only
modes (split, pcie) cannot run here, so this catches a name used in one
mode's result line but defined only in another (the split mode's
median_launch_ms once referenced the frames mode's local)."""
import builtins
import os
import symtable

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _walk(tab, module_names, bad):
    for child in tab.get_children():
        if child.get_type() == "function":
            for sym in child.get_symbols():
                if sym.is_global() and not sym.is_declared_global():
                    name = sym.get_name()
                    if name not in module_names and not hasattr(builtins, name):
                        bad.append(f"{child.get_name()}: {name}")
        _walk(child, module_names, bad)


import pytest

FILES = ["bench.py", "__graft_entry__.py", "gpu-accel-ofdm-ls-mrc_amd/ofdm_lsmrc.py",
         "gpu-accel-ofdm-ls-mrc_amd/antenna_split.py"]


@pytest.mark.parametrize("rel", FILES)
def test_functions_reference_only_defined_names(rel):
    path = os.path.join(ROOT, rel)
    top = symtable.symtable(open(path).read(), path, "exec")
    module_names = {s.get_name() for s in top.get_symbols() if s.is_assigned() or s.is_imported()}
    module_names |= {"__file__", "__name__"}
    bad = []
    _walk(top, module_names, bad)
    assert not bad, f"undefined names in {rel}: {bad}"


def _src(rel):
    with open(os.path.join(ROOT, rel)) as fp:
        return fp.read()


def test_bench_line_carries_box_and_clock_fields():
    """the line shows the box it ran on (same-process HBM
    copy / read ceilings and the effective clock of the timed kernel)."""
    src = _src("bench.py")
    for key in ('"box_copy_GBps"', '"frac_of_box_copy"', '"box_read_GBps"', '"frac_of_box_read"',
                '"clock"', '"effective_GHz_median"', '"per_rank"', '"stages_ms": stages'):
        assert key in src, key


def test_cpu_share_read_from_the_box():
    """no literal CPU share in bench.py."""
    import re
    src = _src("bench.py")
    assert not re.search(r"min\(\s*16\s*,", src)
    assert '"host_cpu_share": 16' not in src
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    share = bench.host_cpu_share()
    assert share["threads"] >= 1 and share["threads"] <= share["affinity_cpus"]
    assert share["source"]


def test_check_failure_invalidates_the_line():
    """a run whose timed output differs from the warm-up's or has
    QPSK errors prints value null with status CHECK_FAILED and exits 1."""
    src = _src("bench.py")
    i = src.index("if failed:  # a broken run")
    block = src[i:i + 400]
    assert '"CHECK_FAILED"' in block and 'result["value"] = None' in block and "sys.exit(1)" in block


def test_stamps_summary_clock():
    """The diagnostic-build stamp records -> effective clock: 2.0 GHz when
    memtime advances 20 ticks per memrealtime tick (100 MHz)."""
    import importlib.util
    import numpy as np
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    rec = np.zeros((4, 12), dtype=np.uint64)
    for i in range(3):
        rec[i] = [1000 + i, 1100 + i, 2000 + i, 50000, 50000 + 20 * 1000, 0, i, i, 0, 0, 0, 0]
    st = bench.stamps_summary(rec)  # the empty 4th record is ignored
    assert st["workgroups"] == 3
    assert abs(st["effective_GHz_median"] - 2.0) < 1e-9
    assert abs(st["stamped_span_ms"] - 1002 * 1e-5) < 1e-12


def test_pmc_traffic_only_for_the_profiled_build(tmp_path):
    """roofline.traffic is attached only from a profile
    whose recorded build id is the running library's (ofdm_lsmrc.build_id);
    a profile of other code gives null and says so."""
    import importlib.util
    import json
    import sys
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    cfg = {"R": 3, "C": 1024, "S": 7, "frames_per_gpu": 5, "prefix": 0, "domain": "time", "flow": "one-launch"}
    p = tmp_path / "t.json"
    with open(p, "w") as fp:
        json.dump({"config": dict(cfg), "mrc_hbm_bytes_per_launch": 123.0, "build_id": "abc"}, fp)
    val, src = bench.pmc_traffic(str(p), cfg, "abc")
    assert val == 123.0 and src.endswith("t.json")
    assert bench.pmc_traffic(str(p), cfg, "def") == (None, "no profile of this build")
    sys.path.insert(0, os.path.join(ROOT, "gpu-accel-ofdm-ls-mrc_amd"))
    import ofdm_lsmrc
    bid = ofdm_lsmrc.build_id()
    assert len(bid) == 16 and int(bid, 16) >= 0 and bid == ofdm_lsmrc.build_id()
    assert '"build_id": build' in _src("bench.py")
    assert '"build_id": bench.get("build_id")' in _src("scripts/pmc_summary.py")
    assert '"build_id": traced.get("build_id")' in _src("scripts/prof_summary_r4.py")
