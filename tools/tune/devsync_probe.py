import time, torch, sys
sys.path.insert(0, "/root/repo")
from elect_amd import _lib
dev = torch.device("cuda", 0)
buf = torch.empty(1 << 31, dtype=torch.uint8, device=dev)
sink = torch.empty(1 << 20, dtype=torch.uint8, device=dev)
s = torch.cuda.Stream(dev)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(1000):
    _lib.hbm_probe(0, buf.data_ptr(), sink.data_ptr(), buf.numel(), stream=s.cuda_stream)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"enqueue {1e3*(t1-t0):.1f} ms, device sync {1e3*(t2-t1):.1f} ms")
