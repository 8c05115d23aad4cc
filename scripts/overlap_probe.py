import sys, time
sys.path.insert(0, 'foveated-rendering-using-ray-tracing_amd')
import fovrt
W, H = 3840, 2160
def mk():
    t = fovrt.PathTracer(fovrt.Config(width=W, height=H, scene=1, mask_mode=4, spp=4, diffuse_max_depth=3))
    t.initialize(); t.update_optix_variables(fovrt.Camera.preset(1, W, H)); return t
a, b = mk(), mk()
for _ in range(3):
    a.frame(False); b.frame(False)
a.synchronize(); b.synchronize()
K = 20
t0 = time.perf_counter()
for _ in range(K): a.frame(False)
a.synchronize(); seq = (time.perf_counter() - t0) / K
t0 = time.perf_counter()
for _ in range(K): a.trace_frame(False)
a.synchronize(); tr = (time.perf_counter() - t0) / K
t0 = time.perf_counter()
for _ in range(K): b.reconstruct_frame(False)
b.synchronize(); rc = (time.perf_counter() - t0) / K
t0 = time.perf_counter()
for _ in range(K):
    a.trace_frame(False); b.reconstruct_frame(False)
a.synchronize(); b.synchronize(); ov = (time.perf_counter() - t0) / K
print(f"sequential frame {seq*1e3:.2f} ms; trace half {tr*1e3:.2f}; recon half {rc*1e3:.2f}; overlapped {ov*1e3:.2f}")
