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
