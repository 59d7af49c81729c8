"""Diagnostic: which candidate pairs pass the bounding-sphere filter (w_pair_near) in gym ur3e-v2
states of main.xml, by geom-type combination -- the compact tier's narrowphase work per forward."""
import collections, ctypes, os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from oracle import pyoracle as po
from ur3e_amd import runtime as rt

md, mc = rt.load_model("main")
n, steps = 64, 120
cfg = rt.make_config(task=rt.TASK_GYM_V2, frame_skip=2, model=md, seed=1, max_episode_steps=100)
ob = po.OracleBatch(mc, po.config_from(cfg), n)
L = po.lib()
L.ur3o_data_geom_pose.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
g1, g2 = np.asarray(md["cpair_geom1"]), np.asarray(md["cpair_geom2"])
rb, mg = np.asarray(md["geom_rbound"]), np.asarray(md["cpair_margin"])
gt = np.asarray(md["geom_type"])
names = {0: "plane", 6: "box", 7: "mesh", 2: "sphere", 5: "cyl", 3: "capsule"}
rng = np.random.default_rng(0)
lo = np.array([0.04799994, -0.11650084, 0.0, 0.0]); hi = np.array([0.54799994, 0.38349916, 0.5, 1.0])
hist, per = collections.Counter(), []
for t in range(steps):
    ob.step(rng.uniform(lo, hi, size=(n, 4)))
    if t % 10 != 9:
        continue
    qp, qv, _, _ = ob.get_state()
    for i in range(0, n, 4):
        d = po.OracleData(mc)
        d.set(qpos=qp[i], qvel=qv[i])
        d.forward()
        xp = np.zeros((md["ngeom"], 3)); xm = np.zeros((md["ngeom"], 9))
        L.ur3o_data_geom_pose(ctypes.byref(mc), d.buf, xp.ctypes.data, xm.ctypes.data)
        dd = np.linalg.norm(xp[g1] - xp[g2], axis=1)
        lim = rb[g1] + rb[g2] + mg
        near = ~((rb[g1] > 0) & (rb[g2] > 0) & (dd > lim))
        per.append(int(near.sum()))
        for p in np.where(near)[0]:
            hist[(names.get(int(gt[g1[p]]), gt[g1[p]]), names.get(int(gt[g2[p]]), gt[g2[p]]), int(g1[p]), int(g2[p]))] += 1
print("candidates", len(g1), "survivors per forward: mean", np.mean(per), "max", max(per), "min", min(per))
for k, v in hist.most_common(30):
    print(k, v / len(per))
