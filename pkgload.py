"""Import helper: the package directory is named ``generic-ebpf_amd`` (not an identifier), so it is
loaded under the module name ``generic_ebpf_amd``."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "generic-ebpf_amd")


def load():
    if "generic_ebpf_amd" in sys.modules:
        return sys.modules["generic_ebpf_amd"]
    spec = importlib.util.spec_from_file_location(
        "generic_ebpf_amd", os.path.join(PKG_DIR, "__init__.py"),
        submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["generic_ebpf_amd"] = mod
    spec.loader.exec_module(mod)
    return mod
