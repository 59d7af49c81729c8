"""GPU: convex mesh geoms (real meshes) bit for bit against the oracle.  The
synthetic scene tests/assets/mesh_scene.xml (committed meshes: STL ASCII/binary, scaled OBJ) exercises
plane-mesh, box-mesh and mesh-mesh contacts; mesh pairs run in the full-capacity tier (GJK/EPA and
plane-convex from ur3e_amd/csrc/convex.h, the oracle's own code), the compact tier hands such env-steps
on.  qpos, qvel, warm start and contact counts must equal the oracle's at every checked step, in the
default two-tier layout and both full-capacity layouts."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ASSETS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets")


@pytest.mark.parametrize("epb", [0, -128, -64])
def test_mesh_scene_bit_exact(epb):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle import pyoracle as po
    from ur3e_amd import runtime as rt
    from ur3e_amd.model.compiler import compile_mjcf, to_ctypes
    md = compile_mjcf(os.path.join(ASSETS, "mesh_scene.xml"))
    assert md["nmesh"] == 3 and 7 in md["geom_type"]
    mc = to_ctypes(md)
    n, steps = 32, 600
    cfg = rt.make_config(task=rt.TASK_CTRL, frame_skip=1, max_episode_steps=0, auto_reset=False, model=md,
                         reset_noise=False, envs_per_block=epb)
    g = rt.Batch(mc, cfg, n)
    ob = po.OracleBatch(mc, po.config_from(cfg), n)
    rng = np.random.default_rng(4)
    q0 = np.tile(np.array(md["qpos0"], float), (n, 1))
    q0[:, 0:2] += rng.uniform(-0.01, 0.01, size=(n, 2))     # mbox xy
    q0[:, 7:9] += rng.uniform(-0.01, 0.01, size=(n, 2))     # prism xy
    q0[:, 2] += rng.uniform(0.0, 0.02, size=n)              # drop heights
    v0 = np.zeros((n, md["nv"]))
    g.set_state(q0, v0)
    ob.set_state(q0, v0)
    kinds = set()
    for t in range(steps):
        a = np.where((t // 150) % 2 == 0, 6.0, -6.0) + rng.uniform(-1, 1, size=(n, 1))
        ob.step(a)
        g.step(torch.from_numpy(a))
        if t % 50 == 0 or t == steps - 1:
            torch.cuda.synchronize()
            qp, qv, wa = g.get_state()
            oqp, oqv, owa, onc = ob.get_state()
            np.testing.assert_array_equal(qp.cpu().numpy(), oqp, err_msg=f"qpos step {t}")
            np.testing.assert_array_equal(qv.cpu().numpy(), oqv, err_msg=f"qvel step {t}")
            np.testing.assert_array_equal(wa.cpu().numpy(), owa, err_msg=f"warm start step {t}")
            np.testing.assert_array_equal(g.get_info()["ncon"].cpu().numpy(), onc, err_msg=f"ncon step {t}")
            kinds |= {tuple(sorted((md["geom_type"][x] for x in pair))) for pair in _oracle_pairs(ob, md)}
    # plane-mesh, box-mesh and mesh-mesh contacts all occurred
    assert {(0, 7), (6, 7), (7, 7)} <= kinds, kinds
    g.close()


def _oracle_pairs(ob, md):
    """geom pairs of the oracle's current contacts over all envs (candidate pairs with ncon > 0)"""
    out = set()
    for i in range(ob.n):
        d = ob.diag(i)
        if d["ncon"] > 0:
            out |= _env_pairs(ob, i)
    return out


def _env_pairs(ob, i):
    import ctypes
    from oracle import pyoracle as po
    sz = ob.L.ur3o_sizeof_env()
    ptr = ctypes.cast(ctypes.addressof(ob.buf) + sz * i, ctypes.c_void_p)
    C = 64
    pos, frame, dist = np.zeros((C, 3)), np.zeros((C, 9)), np.zeros(C)
    geoms, fr, mu, adr = np.zeros((C, 2), np.int32), np.zeros((C, 5)), np.zeros(C), np.zeros(C, np.int32)
    n = ob.L.ur3o_data_contacts(ptr, C, po._p(pos), po._p(frame), po._p(dist), po._p(geoms), po._p(fr), po._p(mu),
                                po._p(adr))
    return {tuple(int(x) for x in geoms[k]) for k in range(min(n, C))}
