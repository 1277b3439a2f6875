import sys, torch
sys.path[:0] = ["/root/repo", "/root/repo/enhanced-unet_amd"]
from eunet import ops
y = torch.randn(4, 1024, 1024, 64, device="cuda").bfloat16()
sc, sh = torch.rand(64, device="cuda"), torch.randn(64, device="cuda")
w, b = torch.randn(2, 64, device="cuda"), torch.randn(2, device="cuda")
z = torch.empty(4, 1024, 1024, 2, device="cuda")
for _ in range(3): ops.bnrelu_conv1x1(ops.act(y), sc, sh, w, b, 2, z)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20): ops.bnrelu_conv1x1(ops.act(y), sc, sh, w, b, 2, z)
e1.record(); torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 20
print(f"bnrelu_conv1x1 4x1024^2x64 bf16: {ms*1e3:.1f} us, {(y.numel()*2 + z.numel()*4)/ms/1e9:.2f} TB/s")
