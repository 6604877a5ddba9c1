"""Is a torch GEMM bit-identical between an eager launch and a HIP-graph replay?"""
import torch

torch.manual_seed(0)
n = 26495
cases = {
    "xT@y [64,n]x[n,64]": (lambda a, b: a.t() @ b, (n, 64), (n, 64)),
    "x@w [n,64]x[64,64]": (lambda a, b: a @ b, (n, 64), (64, 64)),
    "x@wT linear": (lambda a, b: torch.nn.functional.linear(a, b), (n, 64), (64, 64)),
    "gi@Wv [n,64]x[64,4096]": (lambda a, b: a @ b, (n, 64), (64, 4096)),
    "giT@V [64,n]x[n,4096]": (lambda a, b: a.t() @ b, (n, 64), (n, 4096)),
    "sum0": (lambda a, b: a.sum(0), (n, 64), (1,)),
}
for name, (f, sa, sb) in cases.items():
    a = torch.randn(*sa, device="cuda")
    b = torch.randn(*sb, device="cuda")
    e1 = f(a, b).clone()
    e2 = f(a, b).clone()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = f(a, b)
    g.replay()
    torch.cuda.synchronize()
    print(f"{name:28s} eager==eager {torch.equal(e1, e2)}  graph==eager {torch.equal(out, e1)}  "
          f"maxdiff {(out - e1).abs().max().item():.3g}", flush=True)
