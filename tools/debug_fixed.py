import sys, numpy as np, torch
sys.path.insert(0, '/root/repo')
import shorthair_amd as sh
from oracle import pyoracle as po
sh.cauchy_256_init()
for (k, m, B, G) in [(64, 16, 1400, 1), (64, 16, 256, 3), (28, 4, 256, 2), (200, 32, 1400, 2)]:
    d_in = torch.empty((G, k, B), dtype=torch.uint8, device="cuda")
    d_out = torch.zeros((G, m, B), dtype=torch.uint8, device="cuda")
    sh.fill_synthetic(d_in, k, B, G, 0, 7)
    rc = sh.encode_batch(k, m, B, G, d_in, d_out); torch.cuda.synchronize()
    ora = po.oracle()
    for g in range(G):
        data = d_in[g].cpu().numpy()
        _, exp = ora.encode(k, m, data, B)
        got = d_out[g].cpu().numpy()
        bad = np.argwhere(got != exp)
        sub = B // 8
        print(f"k={k} m={m} B={B} g={g} rc={rc} mismatches={len(bad)}/{got.size}")
        if len(bad):
            rows = sorted(set(bad[:, 0].tolist()))
            print("  rows:", rows[:40])
            subs = sorted(set((bad[:, 1] // sub).tolist())); print("  subblocks:", subs)
            cols = sorted(set((bad[:, 1] % sub).tolist())); print("  byte cols (first 20):", cols[:20], "n", len(cols))
            y, p = bad[0]; print("  first: row", y, "byte", p, "got", got[y, p], "exp", exp[y, p])
            print("  row0 got[:8]", got[0, :8], "exp", exp[0, :8])
            print("  zero frac of got:", float((got == 0).mean()))
