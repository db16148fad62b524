"""Which HIP runtimes a process loads, and what each sees (box diagnostics)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pkgload
pkgload.load()
from generic_ebpf_amd import native
order = sys.argv[1] if len(sys.argv) > 1 else "torch"
import torch
if order == "torch":
    print("torch count", torch.cuda.device_count(), flush=True)
    torch.cuda.init()
    print("torch avail", torch.cuda.is_available(), flush=True)
    print("native count", native.gpu_count(), native.last_error(), flush=True)
else:
    print("native count", native.gpu_count(), native.last_error(), flush=True)
    print("torch count", torch.cuda.device_count(), flush=True)
    print("torch avail", torch.cuda.is_available(), flush=True)
for l in open("/proc/self/maps"):
    if "amdhip" in l or "hsa-runtime" in l:
        print(l.split()[-1])
print({k: v for k, v in os.environ.items() if "HIP" in k or "ROC" in k or "HSA" in k or "GPU" in k})
