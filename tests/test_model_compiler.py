"""Model compiler (MJCF subset -> ur3e_model_t) vs facts of the reference models."""
import os

import numpy as np
import pytest

from ur3e_amd.model.compiler import _fk, compile_mjcf, load_json, to_ctypes

ASSETS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ur3e_amd", "assets")


@pytest.mark.parametrize("name,nq,nv,nu,nbody", [("main", 21, 20, 7, 25), ("ur3e_2f85", 14, 14, 7, 23),
                                                 ("ur3e_raw", 6, 6, 6, 8)])
def test_sizes(name, nq, nv, nu, nbody):
    # init_mj.py:36-39 (21/20/7), move_l.py:101-103 (14/14/7), ur3e_raw.xml actuators
    md = load_json(os.path.join(ASSETS, f"{name}.model.json"))
    assert (md["nq"], md["nv"], md["nu"], md["nbody"]) == (nq, nv, nu, nbody)
    to_ctypes(md)  # fits the C image


def test_tcp_kat_and_keyframes():
    md = load_json(os.path.join(ASSETS, "main.model.json"))
    down = np.array(md["key_qpos"][md["id_key_down"]])
    assert down[14:17].tolist() == [0.29799994, 0.13349916, 0.055111]
    xpos, xmat, *_ = _fk(md, down)
    s = md["id_site_tcp"]
    b = md["site_bodyid"][s]
    tcp = xpos[b] + xmat[b] @ np.array(md["site_pos"][s])
    np.testing.assert_allclose(tcp, [0.29799994, 0.13349916, 0.1682003], atol=5e-9)  # main.xml:415


def test_model_physics_constants():
    md = load_json(os.path.join(ASSETS, "main.model.json"))
    # tendon split: 0.5 * right_driver + 0.5 * left_driver (main.xml:349-354)
    assert md["ten_dof"] == [[6, 10]] and md["ten_coef"] == [[0.5, 0.5]]
    # fingers actuator: gain 0.3137255, bias [0, -100, -10], forcerange +-5, ctrlrange [0, 255] (main.xml:381)
    a = 6
    assert md["act_gainprm"][a][0] == 0.3137255 and md["act_biasprm"][a] == [0.0, -100.0, -10.0]
    assert md["act_forcerange"][a] == [-5.0, 5.0] and md["act_ctrlrange"][a] == [0.0, 255.0]
    assert md["act_ctrllimited"] == [1] * 7
    # arm joints: damping 1, frictionloss 0.2 (main.xml:112-142)
    assert md["dof_damping"][:6] == [1.0] * 6 and md["dof_frictionloss"][:6] == [0.2] * 6
    # elliptic cone, impratio 10, dt 1e-3 (main.xml:4)
    assert md["cone"] == 1 and md["impratio"] == 10.0 and md["timestep"] == 0.001
    # explicit pairs present with default pair params
    ex = [k for k in range(md["ncpair"]) if md["cpair_explicit"][k]]
    assert len(ex) == 10
    for k in ex:
        assert md["cpair_friction"][k][:2] == [1.0, 1.0] and md["cpair_solref"][k] == [0.02, 1.0]
    # pad boxes win priority mixing against the fish box
    names = md["geom_names"]
    for k in range(md["ncpair"]):
        g1, g2 = names[md["cpair_geom1"][k]], names[md["cpair_geom2"][k]]
        if {g1, g2} == {"left_pad1", "fish"}:
            assert md["cpair_friction"][k][0] == 0.7 and md["cpair_solref"][k] == [0.004, 1.0]


def test_recompile_matches_committed():
    ref = "/root/reference/assets/main.xml"
    if not os.path.exists(ref):
        pytest.skip("reference not mounted")
    m = compile_mjcf(ref)
    md = load_json(os.path.join(ASSETS, "main.model.json"))
    assert m["ncpair"] == md["ncpair"] and m["cpair_geom1"] == md["cpair_geom1"]
    np.testing.assert_allclose(m["body_invweight0"], md["body_invweight0"], rtol=1e-12)


def test_rest_contacts(main_model):
    """At the 'down' keyframe only the mug touches the table (4 plane-box corners,
    the dist==0 tie of SURVEY H5 is included); no surrogate link overlaps."""
    from oracle import pyoracle as po
    md, mc = main_model
    f = po.forward_state(mc, np.array(md["key_qpos"][md["id_key_down"]]))
    assert f["ncon"] == 4
    f = po.forward_state(mc, np.array(md["key_qpos"][md["id_key_home"]]))
    assert f["ncon"] == 4


def test_generated_main_tree_matches_model():
    """csrc/gen_main_tree.h (compile-time dof tree of the specialised compact kernel) must equal
    the ancestor masks of the shipped main.xml model image."""
    import re
    from ur3e_amd import _build
    path = _build.gen_main_tree()
    txt = open(path).read()
    def arr(name):
        body = re.search(name + r"\[\d+\] = \{([^}]*)\}", txt).group(1)
        return [int(x.strip().rstrip("ul"), 0) for x in body.split(",")]
    masks = arr("ur3e_main_dof_anc_mask")
    md = load_json(os.path.join(ASSETS, "main.model.json"))
    par = md["dof_parentid"][:md["nv"]]
    want = []
    for i in range(md["nv"]):
        m, j = 0, par[i]
        while j >= 0:
            m |= 1 << j
            j = par[j]
        want.append(m)
    assert masks == want
    nb = md["nbody"]
    bpar = md["body_parentid"][:nb]
    assert arr("ur3e_main_body_parent") == bpar
    assert arr("ur3e_main_body_dofnum") == md["body_dofnum"][:nb]
    assert arr("ur3e_main_body_jntadr") == md["body_jntadr"][:nb]
