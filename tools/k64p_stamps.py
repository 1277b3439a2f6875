"""Diagnostic: per-segment clock stamps of the Cin=64 forward kernel (diagnostic build KP_ABL=32).
    EUNET_LIB=abl/libt32.so python tools/k64p_stamps.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "enhanced-unet_amd")]
import torch  # noqa: E402
from eunet import ops  # noqa: E402

N, H, C = 4, int(os.environ.get("H", 1024)), 64
x = torch.randn(N, H, H, C, device="cuda").bfloat16()
w = torch.randn(C, C, 3, 3, device="cuda") / 24
wp = ops.conv3x3_pack(w, torch.bfloat16, flip=False)
y = torch.empty(N, H, H, C, device="cuda", dtype=torch.bfloat16)
tiles = ops.conv3x3_tiles(ops.act(y))
st = torch.zeros(tiles * (2 * C + 1), device="cuda")
sc, sh = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
for _ in range(3):
    ops.conv3x3_fwd(ops.act(x), wp, ops.act(y), bias=torch.zeros(C, device="cuda"), scale=sc, shift=sh, stats=st)
torch.cuda.synchronize()
v = st.view(torch.int64)[: 8 * 8 * 8].view(8, 8, 8).cpu()  # [wave][tile][slot]
names = ["start", "seg1 done", "b1", "seg2 done", "b2", "seg3 done", "b3"]
for wv in (0, 4, 1, 5):
    base = int(v[wv, 0, 0])
    print(f"wave {wv}:")
    for k in range(1, 8):
        row = [int(v[wv, k, s]) - int(v[wv, k, 0]) for s in range(7)]
        print("  tile", k, " ".join(f"{names[s]}={row[s]:6d}" for s in range(1, 7)), " tile_cycles",
              int(v[wv, k, 0]) - int(v[wv, k - 1, 0]))
