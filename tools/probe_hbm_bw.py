"""HBM write / read / copy bandwidth on one MI355X (tooling): fill, sum and copy of large f32
tensors, for the two-pass backward's write-heavy row pass."""
import torch, json
d = torch.device("cuda:0")
n = 4 << 30  # floats = 16 GiB
x = torch.empty(n, dtype=torch.float32, device=d)
y = torch.empty(n // 4, dtype=torch.float32, device=d)
def t(fn, reps=5):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps): fn()
    e.record(); e.synchronize()
    return s.elapsed_time(e) / reps
ms = t(lambda: x.fill_(1.0))
print(json.dumps({"op": "fill 16GiB", "ms": ms, "TBps": 16 * 2**30 / ms / 1e9}))
ms = t(lambda: x.sum())
print(json.dumps({"op": "sum 16GiB", "ms": ms, "TBps": 16 * 2**30 / ms / 1e9}))
z = x[: n // 4]
ms = t(lambda: y.copy_(z))
print(json.dumps({"op": "copy 4GiB", "ms": ms, "TBps": 8 * 2**30 / ms / 1e9}))
