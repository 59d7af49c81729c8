"""Golden vectors for get_site_xrotvec (utils/utils.py:158-162): scipy 1.15.3's
Rotation.from_matrix(xmat).as_rotvec(), run HERE (scipy is importable in this container; nothing from the
reference is imported).  Inputs: random rotations, rotations near identity and near pi about each axis
(each branch of from_matrix's decision and as_rotvec's small-angle series), rounding-level perturbed
matrices (what MuJoCo's site_xmat is), and the tcp xmat of the `down` keyframe.  Writes
tests/golden/rotvec_from_matrix.npz.  usage: python tools/make_rotvec_golden.py"""
import os
import sys

import numpy as np
from scipy.spatial.transform import Rotation as R

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
rng = np.random.default_rng(20261017)
mats = list(R.random(64, random_state=1).as_matrix())
for ax in np.eye(3):
    for ang in (1e-9, 1e-5, 5e-4, 1e-3, 2e-3, 0.5, np.pi - 1e-6, np.pi - 1e-3, np.pi):
        mats.append(R.from_rotvec(ax * ang).as_matrix())
        mats.append(R.from_rotvec(-ax * ang).as_matrix())
for _ in range(16):
    m = R.random(random_state=int(rng.integers(1 << 30))).as_matrix()
    mats.append(m + rng.normal(size=(3, 3)) * 1e-15)
mats.append(np.eye(3))
# the tcp at key `down` (ur3e_env2.py:74 targets rotvec ~ (-1.209, -1.209, 1.209))
from oracle import pyoracle as po
from ur3e_amd import runtime as rt
md, mc = rt.load_model("main")
f = po.forward_state(mc, np.asarray(md["key_qpos"][md["id_key_down"]]))
mats.append(f["site_xmat"][md["id_site_tcp"]].reshape(3, 3))
mats = np.asarray(mats, dtype=np.float64)
rv = np.stack([R.from_matrix(m).as_rotvec() for m in mats])
import scipy
np.savez(os.path.join(REPO, "tests", "golden", "rotvec_from_matrix.npz"), xmat=mats, rotvec=rv,
         scipy_version=np.array(scipy.__version__))
print(len(mats), "matrices; scipy", scipy.__version__)
