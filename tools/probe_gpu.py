"""Minimal GPU probe: libanr_hip.so loads into a torch process and runs on torch's stream."""
import ctypes, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "atmospheric-neural-rendering_amd"))
import torch
import atmonr_amd._lib as L

print("torch", torch.__version__, "hip", torch.version.hip, "gpu", torch.cuda.get_device_name(0), flush=True)
lib = L.load()
dev = torch.device("cuda:0")
s = L.stream(dev)
# sampler
B, N = 4, 8
o = torch.rand(B, 3, device=dev) * 0.1; d = torch.nn.functional.normalize(torch.randn(B, 3, device=dev), dim=1)
ln = torch.full((B,), 0.5, device=dev); u = torch.rand(B, N, device=dev)
bins = torch.linspace(0, 1, N + 1, device=dev)
pts = torch.empty(B, N, 3, device=dev); z = torch.empty(B, N, device=dev)
L.call("anr_sample_uniform_bins", o.data_ptr(), d.data_ptr(), ln.data_ptr(), u.data_ptr(), bins.data_ptr(), B, N, pts.data_ptr(), z.data_ptr(), None, None, s)
zr = (bins[:-1] + u / N) * ln[:, None]; pr = o[:, None] + d[:, None] * zr[..., None]
print("sampler z exact:", torch.equal(z, zr), "pts exact:", torch.equal(pts, pr), flush=True)
# hashgrid
desc = L.hashgrid_desc(3, 16, 2, 16, 1.3819, 19)
table = (torch.rand(desc.n_params, device=dev) * 2e-4 - 1e-4).half()
M = 1 << 20
x = torch.rand(M, 3, device=dev)
out = torch.empty(M, 32, device=dev, dtype=torch.float16)
L.call("anr_hashgrid_fwd", ctypes.byref(desc), x.data_ptr(), 3, M, table.data_ptr(), L.F16, out.data_ptr(), L.F16, 32, s)
torch.cuda.synchronize(); print("hashgrid ok", out.float().abs().mean().item(), flush=True)
g = torch.zeros(desc.n_params, device=dev)
L.call("anr_hashgrid_bwd", ctypes.byref(desc), x.data_ptr(), 3, M, out.data_ptr(), L.F16, 32, g.data_ptr(), s)
torch.cuda.synchronize(); print("hashgrid bwd ok", g.abs().sum().item(), flush=True)
# mlp
md = L.mlp_desc(32, 16, 64, 1, False)
npar = lib.anr_mlp_n_params(ctypes.byref(md))
w = (torch.randn(npar, device=dev) * 0.1)
y = torch.empty(M, 16, device=dev, dtype=torch.float16)
L.call("anr_mlp_fwd", ctypes.byref(md), L.F16, w.half().data_ptr(), out.data_ptr(), L.F16, 32, M, y.data_ptr(), L.F16, 16, s)
torch.cuda.synchronize()
W0 = w[:64*32].view(64, 32); W1 = w[64*32:].view(16, 64)
yr = torch.relu(out[:4096].float() @ W0.half().float().t()) @ W1.half().float().t()
print("mlp fwd max err", (y[:4096].float() - yr).abs().max().item(), "ref scale", yr.abs().max().item(), flush=True)
dw = torch.zeros(npar, device=dev)
dy = torch.randn(M, 16, device=dev)
din = torch.empty(M, 32, device=dev)
L.call("anr_mlp_bwd", ctypes.byref(md), L.F16, w.half().data_ptr(), out.data_ptr(), L.F16, 32, M, dy.data_ptr(), L.F32, 16, din.data_ptr(), L.F32, 32, dw.data_ptr(), s)
torch.cuda.synchronize(); print("mlp bwd ok", dw.abs().sum().item(), din.abs().mean().item(), flush=True)
# timing
for name, fn in [("hash_fwd", lambda: L.call("anr_hashgrid_fwd", ctypes.byref(desc), x.data_ptr(), 3, M, table.data_ptr(), L.F16, out.data_ptr(), L.F16, 32, s)),
                 ("hash_bwd", lambda: L.call("anr_hashgrid_bwd", ctypes.byref(desc), x.data_ptr(), 3, M, out.data_ptr(), L.F16, 32, g.data_ptr(), s)),
                 ("mlp_fwd", lambda: L.call("anr_mlp_fwd", ctypes.byref(md), L.F16, w.half().data_ptr(), out.data_ptr(), L.F16, 32, M, y.data_ptr(), L.F16, 16, s))]:
    fn(); torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(10): fn()
    torch.cuda.synchronize(); print(name, (time.perf_counter() - t) / 10 * 1e3, "ms for M=", M, flush=True)
print("PROBE OK")
