# Gradient error of the MFMA towers vs torch autocast and vs fp32 autograd on
# the same bf16 operands (relative Frobenius, per parameter; rows that differ).
# Output: profiles/r03_mlp_grad_error.log.
import os, sys
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "deeprec-1_amd"))
import deeprec_amd as dr
from deeprec_amd import modelzoo as mz, ops
dr.load()
DEV = "cuda:0"
for sizes in ([13, 512, 256, 128], [479, 512, 256]):
    torch.manual_seed(sum(sizes))
    B = 1024
    mlp = mz._MfmaMLP(sizes, True).to(DEV)
    x = torch.randn((B, sizes[0]), device=DEV, requires_grad=True)
    y = mlp(x); go = torch.randn_like(y); y.backward(go)
    ac = mz._mlp(sizes, True).to(DEV)
    ac.load_state_dict({k.split("net.", 1)[1]: v for k, v in mlp.state_dict().items()})
    xa = x.detach().clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        ya = ac(xa).float()
    ya.backward(go)
    ref = mz._mlp(sizes, True).to(DEV)
    for p, q in zip(ref.parameters(), mlp.net.parameters()):
        with torch.no_grad():
            p.copy_(q.to(torch.bfloat16).float() if p.dim() == 2 else q)
    xr = x.detach().to(torch.bfloat16).float().requires_grad_(True)
    yr = ref(xr); yr.backward(go)
    def rf(a, b): return ((a-b).norm()/b.norm()).item()
    print(sizes, "y ours-ac", rf(y, ya), "ours-fp32", rf(y, yr), "ac-fp32", rf(ya, yr))
    print(" xgrad ours-ac", rf(x.grad, xa.grad), "ours-fp32", rf(x.grad, xr.grad), "ac-fp32", rf(xa.grad, xr.grad))
    rows = ((x.grad - xa.grad).abs().amax(1) > 1e-3).nonzero().flatten()[:10].tolist()
    print(" rows differing ours vs ac:", rows)
    rows = ((x.grad - xr.grad).abs().amax(1) > 2e-2).nonzero().flatten()[:10].tolist()
    print(" rows differing ours vs fp32 (>2e-2):", rows)
    rows = ((xa.grad - xr.grad).abs().amax(1) > 2e-2).nonzero().flatten()[:10].tolist()
    print(" rows differing ac vs fp32 (>2e-2):", rows)
    for (n, p), q, r in zip(ac.named_parameters(), mlp.net.parameters(), ref.parameters()):
        print("  ", n, "ours-ac", round(rf(q.grad, p.grad), 5), "ours-fp32", round(rf(q.grad, r.grad), 5), "ac-fp32", round(rf(p.grad, r.grad), 5))
