"""Dev tool: java train-step loss trajectory with the fused residual+dropout vs torch's x + dropout(o)
(monkeypatched), same init and batches. usage: python tools/loss_ab.py [steps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-structure-aware-transformer_amd"))
import torch  # noqa: E402

import csa_amd.model as M  # noqa: E402
from csa_amd.data import synthetic_batch  # noqa: E402
from csa_amd.train import AdamW, make_train_step  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 15
seeds = [int(a) for a in sys.argv[2:]] or [2021]
dev = torch.device("cuda:0")
fused = M.residual_dropout
batches = [M.batch_to_device(synthetic_batch(64, 150, seed=1 + i), dev) for i in range(3)]
for seed, (name, fn) in ((s, c) for s in seeds for c in (("torch", lambda x, o, d: x + d(o)), ("fused", fused))):
    M.residual_dropout = fn
    torch.manual_seed(seed)
    model = M.CSATrans(**M.CONFIGS["java"]).to(dev)
    opt = AdamW(model.parameters(), lr=1e-4, correct_bias=False)
    step = make_train_step(model, opt, M.label_smoothing_loss, sw=1e-2, scaler=torch.amp.GradScaler("cuda"))
    order = [i % 3 for i in range(5)] + [i % 3 for i in range(steps)]  # bench.py: 5 warm-up, then steps
    losses = [round(float(step(*batches[j])), 4) for j in order]
    print(name, seed, losses, flush=True)
