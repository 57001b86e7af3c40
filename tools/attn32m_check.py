import os, sys, time, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip32, reference as R
dev = "cuda"
def rel(a, b): return float((a.double() - b.double()).norm() / b.double().norm())
for S in (128, 512):
    for p in (0.0, 0.1):
        B, heads = 2, 4; H = heads * 64
        torch.manual_seed(S)
        qkv = torch.randn(B * S, 3 * H, device=dev)
        am = torch.ones(B, S, device=dev); am[1, S - 37:] = 0
        mb = R.key_mask_bias(am)
        g = torch.randn(B * S, H, device=dev)
        res = {}
        for mode in ("m", "v"):
            hip32._ATTN32M = mode == "m"
            a = qkv.clone().requires_grad_()
            out = hip32.attention(a, mb, B, S, heads, p, 1234)
            (out * g).sum().backward()
            res[mode] = (out.detach(), a.grad.detach())
        b = qkv.clone().double().requires_grad_()
        ref = R.attention(b, mb.double(), B, S, heads, p, 1234, p > 0)
        (ref * g.double()).sum().backward()
        for mode in ("m", "v"):
            print(f"S={S} p={p} {mode}: out rel {rel(res[mode][0], ref):.2e}  grad rel {rel(res[mode][1], b.grad):.2e}", flush=True)
# timing at bert-large B=8 S=512
B, S, heads = 8, 512, 16; H = heads * 64
qkv = torch.randn(B * S, 3 * H, device=dev).requires_grad_()
g = torch.randn(B * S, H, device=dev)
for mode in ("m", "v"):
    hip32._ATTN32M = mode == "m"
    for i in range(3):
        out = hip32.attention(qkv, None, B, S, heads, 0.1, 7); out.backward(g)
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for i in range(10):
        out = hip32.attention(qkv, None, B, S, heads, 0.1, 7); out.backward(g)
    torch.cuda.synchronize()
    print(f"bert-large B=8 S=512 fp32 attention fwd+bwd ({mode}): {(time.perf_counter()-t0)/10*1e3:.3f} ms", flush=True)
