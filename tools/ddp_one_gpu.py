"""Multi-rank semantics of the real model on the HIP kernels, on ONE GPU.

Launch (no GPU call happens before the process group exists):
    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 tools/ddp_one_gpu.py [B]

Both ranks run on cuda:0 over the gloo backend (RCCL refuses two ranks on one GPU). Each rank builds the
config/java.py CSATrans with the same deterministic weights, wraps it with csa_amd.train.wrap_ddp (world 2:
the bucketed reducer (16 MB buckets), or torch DDP with CSA_DDP_IMPL=torch (64 MB); the packed QKV parameters, the in-order
attention backward) and runs one eval-mode step (script/train.py:103-116: label-smoothing loss +
sw * sparsity, backward) on its own batch. It then runs the same step on an unwrapped copy of the model on the
same batch and the same Philox seeds, all-gathers those per-rank gradients and checks that DDP's averaged
gradient equals their mean (script/train.py:83 idist.auto_model; SURVEY 8(e): per-rank loss normalisation, so
DDP = the mean of per-rank gradients, not a global-batch gradient). Prints one JSON line on rank 0.
"""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-structure-aware-transformer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    dist.init_process_group("gloo", init_method="env://")  # before any GPU call
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    import golden_inputs as gi  # deterministic parameter fill of the golden fixtures (tests/golden_inputs.py)
    from csa_amd.data import synthetic_batch
    from csa_amd.model import CONFIGS, CSATrans, batch_to_device, label_smoothing_loss
    from csa_amd.train import wrap_ddp

    def build():
        m = CSATrans(**CONFIGS["java"])
        gi.fill_params_deterministic(m, 5)
        return m.to(dev).eval()

    x, y = batch_to_device(synthetic_batch(B, 150, seed=100 + rank), dev)

    def step(model):
        torch.manual_seed(7 + rank)  # the Philox keys of this rank's SBM sampling (_draw_seed)
        out, sp = model(x)[:2]
        loss = label_smoothing_loss(out, y) + 1e-2 * sp
        loss.backward()
        return float(loss.detach())

    t0 = time.time()
    impl = os.environ.get("CSA_DDP_IMPL", "bucketed")
    ddp = wrap_ddp(build(), dev, impl=impl)
    loss_ddp = step(ddp)
    g_ddp = {k: p.grad.detach().clone() for k, p in ddp.module.named_parameters() if p.grad is not None}

    ref = build()
    loss_ref = step(ref)
    g_ref = {k: p.grad.detach() for k, p in ref.named_parameters() if p.grad is not None}
    assert g_ref.keys() == g_ddp.keys()
    worst, nbad = 0.0, 0
    for k in sorted(g_ref):
        parts = [torch.empty_like(g_ref[k]) for _ in range(world)]
        dist.all_gather(parts, g_ref[k].contiguous())
        mean = torch.stack(parts).mean(0)
        d = float((g_ddp[k] - mean).abs().max())
        tol = 1e-6 * float(mean.abs().max()) + 1e-12
        worst = max(worst, d / (float(mean.abs().max()) + 1e-30))
        nbad += d > tol
    losses = [None] * world
    dist.all_gather_object(losses, (loss_ddp, loss_ref))
    if rank == 0:
        print(json.dumps({"test": "DDP (gloo, 2 ranks on cuda:0) gradient == mean of per-rank gradients", "impl": impl,
                          "model": "config/java.py CSATrans (HIP kernels), eval mode", "per_rank_batch": B,
                          "world": world, "tensors": len(g_ref), "tensors_off": int(nbad),
                          "worst_rel_diff": worst, "per_rank_loss_ddp_vs_plain": losses,
                          "seconds": round(time.time() - t0, 1)}), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    if nbad:
        sys.exit(1)


if __name__ == "__main__":
    main()
