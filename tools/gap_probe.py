import sys, os, time, json
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import torch, numpy as np
import bench, util
import sc_polar_decoder_hls_amd as pkg
mask = util.mask("FB_N1024_K512")
dev = torch.device("cuda", 0)
dec = pkg.Decoder(mask); dec.prepare(65536)
llr, _ = bench.gen_frames_torch(torch, mask, 65536, 2.5, 1, dev)
out = torch.empty((65536, dec.words), dtype=torch.int64, device=dev)
st = torch.cuda.current_stream()
for _ in range(5): dec.decode(llr, out, st)
torch.cuda.synchronize()
K = 50
res = {}
# (a) plain launches, events only at both ends
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
t0 = time.perf_counter(); a.record(st)
for _ in range(K): dec.decode(llr, out, st)
b.record(st); torch.cuda.synchronize(); t1 = time.perf_counter()
res["plain_wall_us"] = (t1 - t0) / K * 1e6; res["plain_event_us"] = a.elapsed_time(b) / K * 1e3
# (b) per-step events
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
t0 = time.perf_counter()
for i in range(K):
    ev[i][0].record(st); dec.decode(llr, out, st); ev[i][1].record(st)
torch.cuda.synchronize(); t1 = time.perf_counter()
res["perstep_wall_us"] = (t1 - t0) / K * 1e6; res["perstep_kernel_us"] = float(np.mean([x.elapsed_time(y) for x, y in ev])) * 1e3
# (c) host launch cost alone: time to enqueue K decodes
torch.cuda.synchronize(); t0 = time.perf_counter()
for _ in range(K): dec.decode(llr, out, st)
t1 = time.perf_counter(); torch.cuda.synchronize()
res["enqueue_us"] = (t1 - t0) / K * 1e6
print(json.dumps(res))
