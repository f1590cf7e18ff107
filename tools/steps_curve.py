import importlib, sys, time, subprocess, threading
import torch
sys.path.insert(0, ".")
fm = importlib.import_module("3dgaussian_amd.fit_multiview")
bench = importlib.import_module("bench")
dev = torch.device("cuda:0")
n, V, R = 1_000_000, 50, 800
params = bench.synthetic_params(n, dev)
cams = fm.orbit_cameras(V, R, R, dev)
g = torch.Generator(device=dev).manual_seed(1)
targets = [torch.rand((R, R, 3), generator=g, device=dev) for _ in range(V)]
masks = [(t.mean(dim=2) > 0.5).to(torch.float32) for t in targets]
fit = fm.ViewShardedFitter(params, cams, targets, R, R, lr=0.02, masks=masks)
fit.step(); torch.cuda.synchronize()
clk = []
stop = False
def poll():
    while not stop:
        try:
            out = subprocess.run(["rocm-smi", "--showclocks", "--showpower", "--showtemp"], capture_output=True, text=True, timeout=10).stdout
            clk.append((time.perf_counter(), " | ".join(l.strip() for l in out.splitlines() if ("sclk" in l.lower() or "power" in l.lower() or "junction" in l.lower()) and "GPU[0]" in l)))
        except Exception as e:
            clk.append((time.perf_counter(), str(e)))
        time.sleep(0.5)
th = threading.Thread(target=poll); th.start()
t0 = time.perf_counter(); ts = []
for i in range(120):
    a = time.perf_counter(); fit.step(); torch.cuda.synchronize(); ts.append(time.perf_counter() - a)
stop = True; th.join()
for k in range(0, 120, 10):
    print(f"steps {k:3d}-{k+9:3d}: {1e3*sum(ts[k:k+10])/10:.2f} ms/step")
for t, s in clk[::2]:
    print(f"{t - t0:6.2f}s {s}")
