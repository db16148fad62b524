"""generic-ebpf_amd — MI355X-native batch execution engine for generic-ebpf's eBPF programs.

Python side of the package: instruction encoding (isa), the stepping-aware assembler (layout),
synthetic workloads (workloads) and the ctypes binding of the native C-ABI library
libebpf.so (native).  The hot path itself is native: generic-ebpf_amd/csrc/.
"""
from . import isa, layout, workloads  # noqa: F401
