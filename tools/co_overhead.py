import cProfile, pstats, time, sys, os
sys.path.insert(0, os.getcwd())
import torch, ghex_amd
from ghex_amd.structured import regular as R
N, H = 512, 2
E = N + 2 * H
dev = torch.device("cuda", 0)
base = torch.zeros((E, E, E), dtype=torch.float64, device=dev)
ctx = ghex_amd.make_context()
dd = R.DomainDescriptor(0, (0, 0, 0), (N - 1,) * 3)
pc = R.make_pattern(ctx, R.HaloGenerator((0, 0, 0), (N - 1,) * 3, (H,) * 6, (True,) * 3), [dd])
fd = R.make_field_descriptor(dd, base.permute(2, 1, 0), (H,) * 3, (E,) * 3)
co = R.make_communication_object(ctx)
bis = [pc(fd)]
for _ in range(20):
    co.exchange(bis).wait()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(1000):
    co.exchange(bis).wait()
print("us/exchange", (time.perf_counter() - t) * 1e3)
t = time.perf_counter()
for _ in range(1000):
    co.exchange(bis)
    co._valid = False
torch.cuda.synchronize()
print("us/exchange no wait (queue-bound)", (time.perf_counter() - t) * 1e3)
pr = cProfile.Profile()
pr.enable()
for _ in range(1000):
    co.exchange(bis).wait()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(15)
