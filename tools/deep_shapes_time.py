"""Times the deep shape-only scene of tests/test_gpu_parity.py (thousands of rotated
boxes and ellipsoids) at each register budget of the shape-only fused kernel: the
evidence for api.cpp path_waves' kShapeWavesNodes rule.
    python tools/deep_shapes_time.py [W H spp]"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
import torch  # noqa: E402,F401  (one HIP runtime per process)
from conftest import load_package  # noqa: E402
from test_gpu_parity import deep_shape_scene_text  # noqa: E402

rt = load_package()
W, H, spp = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (960, 540, 16)))
desc, params = rt.parse_scene(deep_shape_scene_text())
params = params.replace(width=W, height=H, spp=spp)
s = rt.Scene(desc)
print("auto", s.tuning(), "nodes", s.info()["bvh_nodes"], "depth", s.info()["bvh_depth"])
for waves in (3, 4, 5):
    s.set_tuning(waves=waves, resume=0)
    s.generate_image(params)
    ks = [s.generate_image(params)[2]["kernel_ms"] for _ in range(3)]
    print(f"waves {waves}: kernel ms {min(ks):.2f} ({', '.join(f'{k:.2f}' for k in ks)})", flush=True)
