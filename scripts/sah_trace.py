import os, sys
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
os.environ["RT_SAH_TRACE"] = "1"
import torch
from synth_scene import make_scene
from skybox_rt_amd import rt
p = make_scene("/tmp/s100k.cgltrace.gz", 100000, seed=3, size=0.012)
s = rt.Scene.load(p)
r = rt.Renderer(s)
r.build_bvh("sah")
print("second build", file=sys.stderr)
st = r.build_bvh("sah")
print(st, file=sys.stderr)
