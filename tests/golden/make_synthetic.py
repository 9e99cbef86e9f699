"""Write the synthetic environment fixtures (no reference data involved).

env_corridor.obj: the snake config's corridor (motionplanningtoolkit_amd.scenes.corridor_env,
seed 0), since snake.inst:16-17 places its only obstacle outside the workspace.
Usage: python tests/golden/make_synthetic.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from motionplanningtoolkit_amd import scenes  # noqa: E402

tris = scenes.corridor_env(0)
out = os.path.join(scenes.MESH_DIR, "env_corridor.obj")
with open(out, "w") as f:
    f.write("# synthetic corridor, motionplanningtoolkit_amd.scenes.corridor_env(seed=0)\no corridor\n")
    for v in tris.reshape(-1, 3):
        f.write("v %.9g %.9g %.9g\n" % tuple(v))
    for t in range(tris.shape[0]):
        f.write("f %d %d %d\n" % (3 * t + 1, 3 * t + 2, 3 * t + 3))
print(out, tris.shape[0])
