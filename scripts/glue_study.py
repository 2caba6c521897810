"""Micro-study of the 5conc bench's client glue: the release token ids gathered from the previous batch's
results into this batch's events (2M random 8-B reads + 2M random 8-B writes), in several torch forms."""
import time
import numpy as np
import torch

N = 4 * 1024 * 1024
dev = torch.device("cuda:0")
rng = np.random.default_rng(1)
perm = rng.permutation(N)
acq = np.sort(perm[: N // 2]); rel = np.sort(perm[N // 2:])
import sys
fifo = len(sys.argv) > 1 and sys.argv[1] == "fifo"
src = acq[rng.permutation(len(acq))[: len(rel)]]
if fifo:                                  # the bench's pairing since round 6: first in, first out
    src = acq[np.sort(rng.permutation(len(acq))[: len(rel)])]
b = torch.zeros((N, 3), dtype=torch.int64, device=dev)
prev = torch.arange(2 * N, dtype=torch.int64, device=dev).view(N, 2)
rel_d = torch.from_numpy(rel.astype(np.int64)).to(dev)
src_d = torch.from_numpy(src.astype(np.int64)).to(dev)
dst_w = rel_d * 3 + 1
src_w = src_d * 2
bf, pf = b.view(-1), prev.view(-1)
# every row's token word from one gather (acquire rows read a zero word appended at the end)
src_all = torch.full((N,), 2 * N, dtype=torch.int64, device=dev)
src_all[rel_d] = src_w
pf = torch.cat([pf, torch.zeros(1, dtype=torch.int64, device=dev)])
variants = {
    "strided index_copy_/index_select": lambda: b[:, 1].index_copy_(0, rel_d, prev[:, 0].index_select(0, src_d)),
    "flat index_copy_/index_select": lambda: bf.index_copy_(0, dst_w, pf.index_select(0, src_w)),
    "flat adv-index assign": lambda: bf.__setitem__(dst_w, pf[src_w]),
    "flat index_put_/take": lambda: bf.index_put_((dst_w,), pf.take(src_w)),
    "flat scatter_/take": lambda: bf.scatter_(0, dst_w, pf.take(src_w)),
    "flat put_/take": lambda: bf.put_(dst_w, pf.take(src_w)),
    "column: gather all rows, strided copy": lambda: b[:, 1].copy_(pf.take(src_all)),
}
ref = None
for name, f in variants.items():
    b.zero_()
    f()
    torch.cuda.synchronize()
    if ref is None:
        ref = b.clone()
    ok = bool(torch.equal(b, ref))
    for _ in range(5):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        f()
    e1.record()
    torch.cuda.synchronize()
    print(f"{name:40s} {e0.elapsed_time(e1) / 50 * 1000:8.1f} us  equal={ok}", flush=True)
