"""Probe: torch's HIP runtime and libcrispr_nw.so in one process, both orders."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
order = sys.argv[1]
if order == "torch_first":
    import torch
    print("torch sees", torch.cuda.device_count(), torch.cuda.is_available(), flush=True)
    x = torch.ones(4, device="cuda:0"); print("torch alloc ok", x.sum().item(), flush=True)
    from crispresso_amd.aligner import GpuAligner
    al = GpuAligner(0); print("aligner ok", flush=True)
else:
    from crispresso_amd.aligner import GpuAligner
    al = GpuAligner(0); print("aligner ok", flush=True)
    import torch
    print("torch sees", torch.cuda.device_count(), torch.cuda.is_available(), flush=True)
    x = torch.ones(4, device="cuda:0"); print("torch alloc ok", x.sum().item(), flush=True)
