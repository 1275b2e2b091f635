import os, sys
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "code-structure-aware-transformer_amd"))
import torch
from torch.profiler import profile, ProfilerActivity
import csa_amd.model as M
dev = torch.device("cuda:0")
gen = M.Generator(20000, 512, 0.2).to(dev).train()
dec = torch.randn(49, 64, 512, device=dev).transpose(0, 1).contiguous().transpose(0, 1).requires_grad_(True)
tgt = torch.randint(1, 20000, (64, 49), device=dev)
scaler = torch.amp.GradScaler("cuda")
for _ in range(2):
    out = gen(dec.permute(1, 0, 2)); loss = M.label_smoothing_loss(out, tgt); scaler.scale(loss).backward()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    out = gen(dec.permute(1, 0, 2)); loss = M.label_smoothing_loss(out, tgt); scaler.scale(loss).backward()
    torch.cuda.synchronize()
for ev in prof.events():
    if ev.name in ("aten::copy_", "aten::clone", "aten::contiguous", "aten::fill_", "aten::zero_") and "20000" in str(ev.input_shapes):
        chain, p = [], ev.cpu_parent
        while p is not None:
            chain.append(p.name); p = p.cpu_parent
        print(ev.name, ev.input_shapes, round(ev.device_time_total, 1), " <- ".join(chain[:5]))
