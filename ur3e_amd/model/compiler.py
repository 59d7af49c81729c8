"""MJCF-subset compiler: reference MJCF -> flat `ur3e_model_t` image.

Replaces `mujoco.MjModel.from_xml_path` (reference `utils/utils.py:9-12`;
`MujocoEnv.__init__` via `gymnasium_env/envs/ur3e_env2.py:32,50-55`) for exactly
the MJCF features the three reference models use:

* `<compiler angle="radian" autolimits="true" meshdir>`, `<option>` (timestep, gravity,
  cone, impratio), `<default>` classes with `class`/`childclass` inheritance;
* bodies (pos, quat), `<inertial>` (diaginertia + quat), hinge and free joints,
  geoms (plane, box, mesh), sites.  Mesh geoms: when every `<asset><mesh>` file exists, real convex
  mesh geoms (`mesh.py`: STL/OBJ, convex hull, MuJoCo's mesh inertia and inertial frame); otherwise
  -- the reference's case, its meshes are git-ignored -- the documented box surrogate
  (`surrogate.py`).  `compile_mjcf(path, meshes="auto" | "mesh" | "surrogate")`;
* `<contact>` `<exclude>` and `<pair>`, fixed tendons, equality connect/joint,
  motor and general(affine) actuators, touch / actuatorfrc / torque sensors, keyframes.

It also performs the `mj_setConst` work MuJoCo does at compile time
(qpos0-based body/dof inverse weights, `meaninertia`, connect anchors in body2's
frame) and the static half of `mj_collision`'s filtering (weld / parent /
contype-conaffinity / exclude / explicit-pair signature), emitting one ordered
collision candidate list with final contact parameters.

The output is a plain dict of numpy arrays (JSON-serialisable) and, through
`to_ctypes`, the C struct declared in `include/ur3e_model.h`.
"""
from __future__ import annotations

import ctypes
import json
import math
import os
import xml.etree.ElementTree as ET

import numpy as np

from . import mesh as _mesh
from .surrogate import DENSITY, MESH_SURROGATE

# ---------------------------------------------------------------------------
# capacities (must equal include/ur3e_model.h)
MAXBODY, MAXJNT, MAXNQ, MAXNV = 28, 16, 24, 24
MAXGEOM, MAXSITE, MAXCPAIR, MAXEQ = 32, 20, 320, 4
MAXU, MAXTEN, MAXTENWRAP, MAXKEY, MAXTOUCH = 8, 2, 4, 2, 4
MAXSENSOR = 16
MAXMESH, MAXMESHVERT = 16, 1024
MODEL_VERSION = 6
SENS_TOUCH, SENS_ACTUATORFRC, SENS_TORQUE = 0, 1, 2

JNT_FREE, JNT_BALL, JNT_SLIDE, JNT_HINGE = 0, 1, 2, 3
GEOM_PLANE, GEOM_BOX, GEOM_MESH = 0, 6, 7
EQ_CONNECT, EQ_JOINT = 0, 2
TRN_JOINT, TRN_TENDON = 0, 3
BIAS_NONE, BIAS_AFFINE = 0, 1

# MuJoCo defaults
DEF_SOLREF = (0.02, 1.0)
DEF_SOLIMP = (0.9, 0.95, 0.001, 0.5, 2.0)
DEF_FRICTION = (1.0, 0.005, 0.0001)


def _floats(s):
    return [float(x) for x in s.split()]


# ---------------------------------------------------------------------------
# small quaternion helpers (w, x, y, z), compile-time only
def qnorm(q):
    q = np.asarray(q, dtype=np.float64)
    n = np.linalg.norm(q)
    return q / n if n > 0 else np.array([1.0, 0, 0, 0])


def qmul(a, b):
    w1, x1, y1, z1 = a
    w2, x2, y2, z2 = b
    return np.array([
        w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2,
        w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
        w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2,
        w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2,
    ])


def q2mat(q):
    w, x, y, z = q
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
        [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
        [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)],
    ])


def mat2q(R):
    # Shepperd; compile-time only (eigenvectors -> body_iquat)
    t = np.trace(R)
    if t > 0:
        s = math.sqrt(t + 1.0) * 2
        q = [0.25 * s, (R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s]
    elif R[0, 0] > R[1, 1] and R[0, 0] > R[2, 2]:
        s = math.sqrt(1.0 + R[0, 0] - R[1, 1] - R[2, 2]) * 2
        q = [(R[2, 1] - R[1, 2]) / s, 0.25 * s, (R[0, 1] + R[1, 0]) / s, (R[0, 2] + R[2, 0]) / s]
    elif R[1, 1] > R[2, 2]:
        s = math.sqrt(1.0 + R[1, 1] - R[0, 0] - R[2, 2]) * 2
        q = [(R[0, 2] - R[2, 0]) / s, (R[0, 1] + R[1, 0]) / s, 0.25 * s, (R[1, 2] + R[2, 1]) / s]
    else:
        s = math.sqrt(1.0 + R[2, 2] - R[0, 0] - R[1, 1]) * 2
        q = [(R[1, 0] - R[0, 1]) / s, (R[0, 2] + R[2, 0]) / s, (R[1, 2] + R[2, 1]) / s, 0.25 * s]
    return qnorm(q)


# ---------------------------------------------------------------------------
class _Defaults:
    """MJCF default-class tree: class name -> {element tag -> {attr: value}}."""

    def __init__(self, root):
        self.cls = {"main": {}}
        self.parent = {"main": None}
        d = root.find("default")
        if d is not None:
            self._walk(d, "main")

    def _walk(self, node, name):
        for ch in node:
            if ch.tag == "default":
                cname = ch.get("class")
                self.parent[cname] = name
                self.cls[cname] = {}
                self._walk(ch, cname)
            else:
                self.cls[name].setdefault(ch.tag, {}).update(ch.attrib)

    def resolve(self, tag, cname):
        chain = []
        c = cname
        while c is not None:
            chain.append(c)
            c = self.parent[c]
        out = {}
        for c in reversed(chain):
            out.update(self.cls[c].get(tag, {}))
        return out


def _attrs(defaults, el, childclass):
    cname = el.get("class") or childclass or "main"
    tag = el.tag
    # actuator shortcuts share the 'general' defaults in MuJoCo for affine params
    a = defaults.resolve(tag, cname)
    if tag == "motor":
        a = dict(a)
    a.update({k: v for k, v in el.attrib.items() if k != "class"})
    return a


# ---------------------------------------------------------------------------
def _mesh_assets(root, defaults, path, meshdir_override=None):
    """<asset><mesh> entries: name -> {file (resolved against <compiler meshdir>, or against
    meshdir_override when given), scale, inertia}"""
    comp = root.find("compiler")
    meshdir = comp.get("meshdir", "") if comp is not None else ""
    base = os.path.join(os.path.dirname(os.path.abspath(path)), meshdir)
    if meshdir_override is not None:
        base = meshdir_override
    out = {}
    asset = root.find("asset")
    if asset is None:
        return out
    for ch in asset:
        if ch.tag != "mesh":
            continue
        a = dict(defaults.resolve("mesh", ch.get("class") or "main"))
        a.update({k: v for k, v in ch.attrib.items() if k != "class"})
        f = a["file"]
        name = a.get("name") or os.path.splitext(os.path.basename(f))[0]
        out[name] = dict(file=os.path.join(base, f), scale=(_floats(a.get("scale", "1 1 1")) + [1.0] * 3)[:3],
                         inertia=a.get("inertia", "legacy"))
    return out


def compile_mjcf(path: str, meshes: str = "auto", meshdir: str | None = None) -> dict:
    """Compile one MJCF file into a model dict.  meshes: "auto" = real mesh geoms when every mesh file
    exists, else the box surrogate; "mesh" = real meshes (missing files raise); "surrogate".
    meshdir: resolve the mesh files against this directory instead of the MJCF's <compiler meshdir>
    (the same relative file names), e.g. a directory of substitute meshes."""
    tree = ET.parse(path)
    root = tree.getroot()
    defaults = _Defaults(root)
    model_name = os.path.basename(path)
    if meshes not in ("auto", "mesh", "surrogate"):
        raise ValueError(f"meshes must be 'auto', 'mesh' or 'surrogate', got {meshes!r}")
    assets = _mesh_assets(root, defaults, path, meshdir)
    missing = [a["file"] for a in assets.values() if not os.path.exists(a["file"])]
    if meshes == "mesh" and missing:
        raise FileNotFoundError(f"mesh files missing: {missing}")
    real_meshes = bool(assets) and not missing and meshes != "surrogate"
    mesh_cache = {}

    comp = root.find("compiler")
    autolimits = comp is not None and comp.get("autolimits", "false") == "true"
    if comp is not None and comp.get("angle", "degree") != "radian":
        raise ValueError("only angle='radian' models are supported")

    opt = root.find("option")
    timestep = 0.002
    gravity = [0.0, 0.0, -9.81]
    cone = 0
    impratio = 1.0
    if opt is not None:
        timestep = float(opt.get("timestep", timestep))
        if opt.get("gravity"):
            gravity = _floats(opt.get("gravity"))
        cone = 1 if opt.get("cone", "pyramidal") == "elliptic" else 0
        impratio = float(opt.get("impratio", 1.0))

    bodies = []   # dicts
    joints = []
    geoms = []    # all geoms incl. visual (for inertia)
    sites = []
    names = {"body": {}, "joint": {}, "geom": {}, "site": {}}

    bodies.append(dict(name="world", parent=-1, pos=np.zeros(3), quat=np.array([1.0, 0, 0, 0]),
                       inertial=None, joints=[], geoms=[], sites=[], childclass=None))
    names["body"]["world"] = 0

    def walk(el, parent_id, childclass):
        for ch in el:
            if ch.tag == "body":
                bid = len(bodies)
                cc = ch.get("childclass") or childclass
                b = dict(name=ch.get("name", f"body{bid}"), parent=parent_id,
                         pos=np.array(_floats(ch.get("pos", "0 0 0"))),
                         quat=qnorm(_floats(ch.get("quat", "1 0 0 0"))),
                         inertial=None, joints=[], geoms=[], sites=[], childclass=cc)
                bodies.append(b)
                names["body"][b["name"]] = bid
                _body_content(ch, bid, cc)
                walk(ch, bid, cc)
            elif ch.tag in ("geom", "site") and parent_id == 0:
                pass  # handled by _body_content(world)

    def _body_content(el, bid, cc):
        b = bodies[bid]
        for ch in el:
            if ch.tag == "inertial":
                b["inertial"] = dict(pos=np.array(_floats(ch.get("pos", "0 0 0"))),
                                     quat=qnorm(_floats(ch.get("quat", "1 0 0 0"))),
                                     mass=float(ch.get("mass")),
                                     diag=np.array(_floats(ch.get("diaginertia"))))
            elif ch.tag in ("joint", "freejoint"):
                a = _attrs(defaults, ch, cc) if ch.tag == "joint" else {"type": "free"}
                jt = a.get("type", "hinge")
                jtype = {"free": JNT_FREE, "ball": JNT_BALL, "slide": JNT_SLIDE, "hinge": JNT_HINGE}[jt]
                rng = _floats(a["range"]) if "range" in a else [0.0, 0.0]
                if "limited" in a:
                    limited = a["limited"] == "true"
                else:
                    limited = autolimits and "range" in a
                j = dict(name=a.get("name", f"jnt{len(joints)}"), body=bid, type=jtype,
                         pos=np.array(_floats(a.get("pos", "0 0 0"))),
                         axis=qnorm([0.0] + _floats(a.get("axis", "0 0 1")))[1:] if jtype != JNT_FREE
                         else np.array([0.0, 0.0, 1.0]),
                         range=rng, limited=int(limited and jtype != JNT_FREE),
                         stiffness=float(a.get("stiffness", 0.0)),
                         springref=float(a.get("springref", 0.0)),
                         damping=float(a.get("damping", 0.0)),
                         armature=float(a.get("armature", 0.0)),
                         frictionloss=float(a.get("frictionloss", 0.0)),
                         margin=float(a.get("margin", 0.0)),
                         solreflimit=_floats(a["solreflimit"]) if "solreflimit" in a else list(DEF_SOLREF),
                         solimplimit=_pad_solimp(_floats(a["solimplimit"])) if "solimplimit" in a
                         else list(DEF_SOLIMP),
                         solreffriction=_floats(a["solreffriction"]) if "solreffriction" in a
                         else list(DEF_SOLREF),
                         solimpfriction=_pad_solimp(_floats(a["solimpfriction"])) if "solimpfriction" in a
                         else list(DEF_SOLIMP))
                names["joint"][j["name"]] = len(joints)
                joints.append(j)
                b["joints"].append(len(joints) - 1)
            elif ch.tag == "geom":
                a = _attrs(defaults, ch, cc)
                g = _make_geom(a, bid, assets if real_meshes else None, mesh_cache)
                if ch.get("name"):
                    names["geom"][ch.get("name")] = len(geoms)
                g["name"] = ch.get("name")
                geoms.append(g)
                b["geoms"].append(len(geoms) - 1)
            elif ch.tag == "site":
                a = _attrs(defaults, ch, cc)
                s = dict(name=a.get("name", f"site{len(sites)}"), body=bid,
                         type={"sphere": 2, "capsule": 3, "ellipsoid": 4, "cylinder": 5, "box": 6}.get(
                             a.get("type", "sphere"), 2),
                         pos=np.array(_floats(a.get("pos", "0 0 0"))),
                         quat=qnorm(_floats(a.get("quat", "1 0 0 0"))),
                         size=(_floats(a.get("size", "0.005")) + [0.0, 0.0, 0.0])[:3])
                names["site"][s["name"]] = len(sites)
                sites.append(s)
                b["sites"].append(len(sites) - 1)

    wb = root.find("worldbody")
    _body_content(wb, 0, None)
    walk(wb, 0, None)

    nbody = len(bodies)
    if nbody > MAXBODY:
        raise ValueError("too many bodies")

    # ---------------- body tree bookkeeping
    parent = [b["parent"] for b in bodies]
    rootid = [0] * nbody
    for i in range(1, nbody):
        rootid[i] = i if parent[i] == 0 else rootid[parent[i]]
    weldid = [0] * nbody
    for i in range(1, nbody):
        weldid[i] = i if bodies[i]["joints"] else weldid[parent[i]]

    # ---------------- joints / dofs (joints are already in depth-first order)
    njnt = len(joints)
    qposadr, dofadr = [], []
    nq = nv = 0
    dof_body, dof_jnt = [], []
    for ji, j in enumerate(joints):
        qposadr.append(nq)
        dofadr.append(nv)
        if j["type"] == JNT_FREE:
            nq += 7
            nv += 6
            ndof = 6
        elif j["type"] == JNT_BALL:
            nq += 4
            nv += 3
            ndof = 3
        else:
            nq += 1
            nv += 1
            ndof = 1
        for _ in range(ndof):
            dof_body.append(j["body"])
            dof_jnt.append(ji)
    body_jntnum = [len(b["joints"]) for b in bodies]
    body_jntadr = [b["joints"][0] if b["joints"] else -1 for b in bodies]
    body_dofnum = [0] * nbody
    body_dofadr = [-1] * nbody
    for d, bid in enumerate(dof_body):
        if body_dofadr[bid] < 0:
            body_dofadr[bid] = d
        body_dofnum[bid] += 1
    # dof_parentid
    last_dof = [-1] * nbody
    dof_parent = [-1] * nv
    for i in range(1, nbody):
        p = last_dof[parent[i]]
        for k in range(body_dofnum[i]):
            d = body_dofadr[i] + k
            dof_parent[d] = p
            p = d
        last_dof[i] = p

    qpos0 = np.zeros(nq)
    qpos_spring = np.zeros(nq)
    for ji, j in enumerate(joints):
        a = qposadr[ji]
        if j["type"] == JNT_FREE:
            b = bodies[j["body"]]
            qpos0[a:a + 3] = b["pos"]
            qpos0[a + 3:a + 7] = b["quat"]
            qpos_spring[a:a + 7] = qpos0[a:a + 7]
        else:
            qpos0[a] = 0.0
            qpos_spring[a] = j["springref"]

    # ---------------- inertia (explicit or from geoms)
    body_mass = np.zeros(nbody)
    body_ipos = np.zeros((nbody, 3))
    body_iquat = np.tile([1.0, 0, 0, 0], (nbody, 1))
    body_inertia = np.zeros((nbody, 3))
    for i, b in enumerate(bodies):
        if i == 0:
            continue
        if b["inertial"] is not None:
            body_mass[i] = b["inertial"]["mass"]
            body_ipos[i] = b["inertial"]["pos"]
            body_iquat[i] = b["inertial"]["quat"]
            body_inertia[i] = b["inertial"]["diag"]
        else:
            m, ipos, iquat, inert = _inertia_from_geoms([geoms[g] for g in b["geoms"]])
            body_mass[i], body_ipos[i], body_iquat[i], body_inertia[i] = m, ipos, iquat, inert
    subtreemass = body_mass.copy()
    for i in range(nbody - 1, 0, -1):
        subtreemass[parent[i]] += subtreemass[i]

    # ---------------- collision geoms
    col = [gi for gi, g in enumerate(geoms) if (g["contype"] or g["conaffinity"])]
    if len(col) > MAXGEOM:
        raise ValueError("too many collision geoms")
    colidx = {gi: k for k, gi in enumerate(col)}

    # ---------------- contact pairs / excludes
    contact = root.find("contact")
    excludes = set()
    explicit = []
    if contact is not None:
        for ch in contact:
            if ch.tag == "exclude":
                b1 = names["body"][ch.get("body1")]
                b2 = names["body"][ch.get("body2")]
                excludes.add((min(b1, b2), max(b1, b2)))
            elif ch.tag == "pair":
                a = _attrs(defaults, ch, None)
                g1 = names["geom"][a["geom1"]]
                g2 = names["geom"][a["geom2"]]
                explicit.append((g1, g2, a))

    def sig(g1, g2):
        b1, b2 = geoms[g1]["body"], geoms[g2]["body"]
        return (min(b1, b2) << 16) + max(b1, b2)

    explicit_sigs = set(sig(g1, g2) for g1, g2, _ in explicit)
    cands = []
    for g1, g2, a in explicit:
        if g1 not in colidx or g2 not in colidx:
            # an explicit pair with a non-colliding (visual) geom still collides in MuJoCo;
            # surrogate non-colliding meshes are dropped here and logged.
            continue
        if geoms[g1]["type"] > geoms[g2]["type"]:
            g1, g2 = g2, g1
        p = _mix_params(geoms[g1], geoms[g2])
        # explicit attributes override the mixed values
        if "condim" in a:
            p["condim"] = int(a["condim"])
        if "friction" in a:
            p["friction"] = (_floats(a["friction"]) + [0.0] * 5)[:5]
        if "solref" in a:
            p["solref"] = _floats(a["solref"])
        if "solimp" in a:
            p["solimp"] = _pad_solimp(_floats(a["solimp"]))
        if "margin" in a:
            p["margin"] = float(a["margin"])
        if "gap" in a:
            p["gap"] = float(a["gap"])
        cands.append((sig(g1, g2), 0, g1, g2, 1, p))
    for ia in range(len(col)):
        for ib in range(ia + 1, len(col)):
            g1, g2 = col[ia], col[ib]
            b1, b2 = geoms[g1]["body"], geoms[g2]["body"]
            w1, w2 = weldid[b1], weldid[b2]
            if w1 == w2:
                continue
            pw1, pw2 = weldid[parent[w1]] if w1 else 0, weldid[parent[w2]] if w2 else 0
            if w1 != 0 and w2 != 0 and (w1 == pw2 or w2 == pw1):
                continue
            ga, gb = geoms[g1], geoms[g2]
            if not ((ga["contype"] & gb["conaffinity"]) or (gb["contype"] & ga["conaffinity"])):
                continue
            if (min(b1, b2), max(b1, b2)) in excludes:
                continue
            s = sig(g1, g2)
            if s in explicit_sigs:
                continue
            if ga["type"] == GEOM_PLANE and gb["type"] == GEOM_PLANE:
                continue
            if ga["type"] > gb["type"]:
                g1, g2 = g2, g1
            cands.append((s, 1, g1, g2, 0, _mix_params(geoms[g1], geoms[g2])))
    cands.sort(key=lambda c: (c[0], c[1], c[2], c[3]))
    if len(cands) > MAXCPAIR:
        raise ValueError(f"too many collision candidates: {len(cands)}")

    # ---------------- tendons
    tendons = []
    ten = root.find("tendon")
    if ten is not None:
        for ch in ten:
            if ch.tag == "fixed":
                wr = []
                for w in ch:
                    ji = names["joint"][w.get("joint")]
                    wr.append((dofadr[ji], float(w.get("coef", 1.0))))
                tendons.append(dict(name=ch.get("name"), wraps=wr))
    ten_names = {t["name"]: i for i, t in enumerate(tendons)}

    # ---------------- actuators
    acts = []
    ac = root.find("actuator")
    if ac is not None:
        for ch in ac:
            cc = None
            a = defaults.resolve("general", ch.get("class") or "main") if ch.tag == "general" else {}
            a = dict(a)
            if ch.tag == "motor":
                a.update(defaults.resolve("motor", ch.get("class") or "main"))
            a.update({k: v for k, v in ch.attrib.items() if k != "class"})
            if "joint" in a:
                trntype, trnid = TRN_JOINT, names["joint"][a["joint"]]
            elif "tendon" in a:
                trntype, trnid = TRN_TENDON, ten_names[a["tendon"]]
            else:
                raise ValueError("unsupported actuator transmission")
            if ch.tag == "motor":
                gain, biastype, bias = [1.0, 0, 0], BIAS_NONE, [0.0, 0, 0]
            else:
                gain = (_floats(a.get("gainprm", "1")) + [0.0] * 3)[:3]
                bt = a.get("biastype", "none")
                biastype = BIAS_AFFINE if bt == "affine" else BIAS_NONE
                bias = (_floats(a.get("biasprm", "0")) + [0.0] * 3)[:3]
            cr = _floats(a["ctrlrange"]) if "ctrlrange" in a else [0.0, 0.0]
            fr = _floats(a["forcerange"]) if "forcerange" in a else [0.0, 0.0]
            if "ctrllimited" in a:
                cl = a["ctrllimited"] == "true"
            else:
                cl = autolimits and "ctrlrange" in a
            if "forcelimited" in a:
                fl = a["forcelimited"] == "true"
            else:
                fl = autolimits and "forcerange" in a
            acts.append(dict(name=a.get("name"), trntype=trntype, trnid=trnid, gain=gain,
                             biastype=biastype, bias=bias, ctrlrange=cr, forcerange=fr,
                             ctrllimited=int(cl), forcelimited=int(fl),
                             gear=float(_floats(a.get("gear", "1"))[0])))
    nu = len(acts)

    # ---------------- equality
    eqs = []
    eqel = root.find("equality")
    if eqel is not None:
        for ch in eqel:
            a = _attrs(defaults, ch, None)
            solref = _floats(a["solref"]) if "solref" in a else list(DEF_SOLREF)
            solimp = _pad_solimp(_floats(a["solimp"])) if "solimp" in a else list(DEF_SOLIMP)
            data = np.zeros(11)
            if ch.tag == "connect":
                o1 = names["body"][a["body1"]]
                o2 = names["body"][a.get("body2", "world")]
                data[0:3] = _floats(a.get("anchor", "0 0 0"))
                eqs.append(dict(type=EQ_CONNECT, obj1=o1, obj2=o2, data=data, solref=solref, solimp=solimp))
            elif ch.tag == "joint":
                o1 = names["joint"][a["joint1"]]
                o2 = names["joint"][a["joint2"]] if "joint2" in a else -1
                pc = (_floats(a.get("polycoef", "0 1 0 0 0")) + [0.0] * 5)[:5]
                data[0:5] = pc
                eqs.append(dict(type=EQ_JOINT, obj1=o1, obj2=o2, data=data, solref=solref, solimp=solimp))
            else:
                raise ValueError(f"unsupported equality {ch.tag}")

    # ---------------- sensors, in declaration order (mjData.sensordata layout): touch (1 value, site),
    # actuatorfrc (1, actuator), torque (3, site; needs mj_rnePostConstraint)
    touch = []
    sens_type, sens_obj, sens_adr = [], [], []
    act_names = {a["name"]: k for k, a in enumerate(acts)}
    nsd = 0
    se = root.find("sensor")
    if se is not None:
        for ch in se:
            if not isinstance(ch.tag, str):
                continue
            if ch.tag == "touch":
                obj = names["site"][ch.get("site")]
                touch.append(obj)
                t, dim = SENS_TOUCH, 1
            elif ch.tag == "actuatorfrc":
                obj, t, dim = act_names[ch.get("actuator")], SENS_ACTUATORFRC, 1
            elif ch.tag == "torque":
                obj, t, dim = names["site"][ch.get("site")], SENS_TORQUE, 3
            else:
                raise ValueError(f"unsupported sensor {ch.tag}")
            sens_type.append(t)
            sens_obj.append(obj)
            sens_adr.append(nsd)
            nsd += dim

    # ---------------- convex meshes of the collision geoms: one hull per mesh asset, pooled
    mesh_names, mesh_adr, mesh_num, mesh_vert = [], [], [], []
    geom_dataid = []
    for gi in col:
        g = geoms[gi]
        if g["type"] != GEOM_MESH:
            geom_dataid.append(-1)
            continue
        if g["mesh"] not in mesh_names:
            mesh_names.append(g["mesh"])
            mesh_adr.append(len(mesh_vert))
            mesh_num.append(len(g["hull"]))
            mesh_vert.extend(np.asarray(g["hull"]).tolist())
        geom_dataid.append(mesh_names.index(g["mesh"]))
    if len(mesh_names) > MAXMESH or len(mesh_vert) > MAXMESHVERT:
        raise ValueError(f"convex meshes exceed the model image ({len(mesh_names)} meshes, {len(mesh_vert)} hull "
                         f"vertices; capacities {MAXMESH}, {MAXMESHVERT})")

    # ---------------- keyframes
    keys = {}
    ke = root.find("keyframe")
    if ke is not None:
        for ch in ke:
            q = np.array(_floats(ch.get("qpos"))) if ch.get("qpos") else qpos0.copy()
            v = np.array(_floats(ch.get("qvel"))) if ch.get("qvel") else np.zeros(nv)
            keys[ch.get("name")] = (q, v)
    key_names = list(keys.keys())

    m = dict(
        name=model_name, version=MODEL_VERSION,
        nq=nq, nv=nv, nu=nu, nbody=nbody, njnt=njnt, ngeom=len(col), nsite=len(sites),
        ncpair=len(cands), neq=len(eqs), ntendon=len(tendons), nkey=len(key_names), ntouch=len(touch),
        timestep=timestep, gravity=gravity, cone=cone, impratio=impratio,
        tolerance=1e-8, iterations=100, ls_iterations=50, ls_tolerance=0.01,
        body_parentid=parent, body_rootid=rootid, body_weldid=weldid,
        body_jntnum=body_jntnum, body_jntadr=body_jntadr, body_dofnum=body_dofnum, body_dofadr=body_dofadr,
        body_pos=[b["pos"].tolist() for b in bodies], body_quat=[b["quat"].tolist() for b in bodies],
        body_ipos=body_ipos.tolist(), body_iquat=body_iquat.tolist(), body_mass=body_mass.tolist(),
        body_subtreemass=subtreemass.tolist(), body_inertia=body_inertia.tolist(),
        jnt_type=[j["type"] for j in joints], jnt_qposadr=qposadr, jnt_dofadr=dofadr,
        jnt_bodyid=[j["body"] for j in joints], jnt_limited=[j["limited"] for j in joints],
        jnt_pos=[j["pos"].tolist() for j in joints], jnt_axis=[list(map(float, j["axis"])) for j in joints],
        jnt_range=[list(j["range"]) for j in joints], jnt_stiffness=[j["stiffness"] for j in joints],
        jnt_margin=[j["margin"] for j in joints], jnt_solref=[j["solreflimit"] for j in joints],
        jnt_solimp=[j["solimplimit"] for j in joints],
        dof_bodyid=dof_body, dof_jntid=dof_jnt, dof_parentid=dof_parent,
        dof_armature=[joints[j]["armature"] for j in dof_jnt],
        dof_damping=[joints[j]["damping"] for j in dof_jnt],
        dof_frictionloss=[joints[j]["frictionloss"] for j in dof_jnt],
        dof_solref=[joints[j]["solreffriction"] for j in dof_jnt],
        dof_solimp=[joints[j]["solimpfriction"] for j in dof_jnt],
        qpos0=qpos0.tolist(), qpos_spring=qpos_spring.tolist(),
        geom_type=[geoms[g]["type"] for g in col], geom_bodyid=[geoms[g]["body"] for g in col],
        geom_surrogate=[geoms[g]["surrogate"] for g in col],
        geom_pos=[geoms[g]["pos"].tolist() for g in col], geom_quat=[geoms[g]["quat"].tolist() for g in col],
        geom_size=[list(geoms[g]["size"]) for g in col],
        geom_rbound=[geoms[g]["rbound"] for g in col],
        geom_names=[geoms[g]["name"] for g in col],
        site_bodyid=[s["body"] for s in sites], site_type=[s["type"] for s in sites],
        site_pos=[s["pos"].tolist() for s in sites], site_quat=[s["quat"].tolist() for s in sites],
        site_size=[list(s["size"]) for s in sites], site_names=[s["name"] for s in sites],
        cpair_geom1=[colidx[c[2]] for c in cands], cpair_geom2=[colidx[c[3]] for c in cands],
        cpair_explicit=[c[4] for c in cands], cpair_condim=[c[5]["condim"] for c in cands],
        cpair_friction=[c[5]["friction"] for c in cands], cpair_solref=[c[5]["solref"] for c in cands],
        cpair_solimp=[c[5]["solimp"] for c in cands], cpair_margin=[c[5]["margin"] for c in cands],
        cpair_gap=[c[5]["gap"] for c in cands],
        ten_num=[len(t["wraps"]) for t in tendons], ten_dof=[[w[0] for w in t["wraps"]] for t in tendons],
        ten_coef=[[w[1] for w in t["wraps"]] for t in tendons],
        eq_type=[e["type"] for e in eqs], eq_obj1=[e["obj1"] for e in eqs], eq_obj2=[e["obj2"] for e in eqs],
        eq_data=[e["data"].tolist() for e in eqs], eq_solref=[e["solref"] for e in eqs],
        eq_solimp=[e["solimp"] for e in eqs],
        act_trntype=[a["trntype"] for a in acts], act_trnid=[a["trnid"] for a in acts],
        act_gaintype=[0] * nu, act_biastype=[a["biastype"] for a in acts],
        act_ctrllimited=[a["ctrllimited"] for a in acts], act_forcelimited=[a["forcelimited"] for a in acts],
        act_ctrlrange=[a["ctrlrange"] for a in acts], act_forcerange=[a["forcerange"] for a in acts],
        act_gainprm=[a["gain"] for a in acts], act_biasprm=[a["bias"] for a in acts],
        act_gear=[a["gear"] for a in acts], act_names=[a["name"] for a in acts],
        touch_site=touch,
        nsensor=len(sens_type), nsensordata=nsd, sensor_type=sens_type, sensor_objid=sens_obj,
        sensor_adr=sens_adr,
        key_names=key_names,
        key_qpos=[keys[k][0].tolist() for k in key_names], key_qvel=[keys[k][1].tolist() for k in key_names],
        body_names=[b["name"] for b in bodies], joint_names=[j["name"] for j in joints],
        nmesh=len(mesh_names), nmeshvert=len(mesh_vert), geom_dataid=geom_dataid, mesh_vertadr=mesh_adr,
        mesh_vertnum=mesh_num, mesh_vert=mesh_vert, mesh_names=mesh_names,
    )

    def _nid(kind, nm):
        return names[kind].get(nm, -1)

    m["id_site_tcp"] = _nid("site", "tcp")
    m["id_site_handle"] = _nid("site", "handle_site")
    m["id_site_lpad"] = _nid("site", "left_pad1_site")
    m["id_site_rpad"] = _nid("site", "right_pad1_site")
    m["id_body_fish"] = _nid("body", "fish")
    m["id_body_ghost"] = _nid("body", "ghost")
    m["id_body_lpad"] = _nid("body", "left_pad")
    m["id_body_rpad"] = _nid("body", "right_pad")
    m["id_body_table"] = _nid("body", "table")
    m["id_key_home"] = key_names.index("home") if "home" in key_names else -1
    m["id_key_down"] = key_names.index("down") if "down" in key_names else -1

    def _subtree_mask(rootname):
        r = names["body"].get(rootname, -1)
        if r < 0:
            return 0
        mask = 0
        for i in range(nbody):
            j = i
            while j > 0 and j != r:
                j = parent[j]
            if j == r:
                mask |= 1 << i
        return mask

    arm_root = "robot_base" if "robot_base" in names["body"] else "base"
    m["mask_arm_bodies"] = _subtree_mask(arm_root)
    m["mask_gripper_bodies"] = _subtree_mask("robotiq_base_mount")
    fish = m["id_body_fish"]
    if fish >= 0:
        fg = [g for g in geoms if g["body"] == fish][0]
        m["fish_topple_z"] = max(fg["size"][0], fg["size"][1])
        m["fish_half_z"] = fg["size"][2]  # get_body_size(m, "fish")[-1] (ur3e_env.py compute_reward)
    else:
        m["fish_topple_z"] = 0.0
        m["fish_half_z"] = 0.0

    _set_const(m)
    return m


def _pad_solimp(v):
    v = list(v) + list(DEF_SOLIMP[len(v):])
    return v[:5]


def _load_convex(asset, cache):
    """mesh asset -> hull vertices in the mesh's inertial frame, unit-density volume and principal
    inertia, and that frame (com, rotation) in mesh coordinates (mjCMesh processing)"""
    key = asset["file"], tuple(asset["scale"]), asset["inertia"]
    if key not in cache:
        v, f = _mesh.load_mesh(asset["file"], asset["scale"])
        hidx, _ = _mesh.convex_hull(v)
        vol, com, I = _mesh.mesh_inertia(v, f, asset["inertia"])
        w, Rp = _mesh.principal_frame(I)
        hull = (v[hidx] - com) @ Rp  # coordinates along the principal axes
        cache[key] = dict(hull=hull, vol=vol, inertia=w, com=com, R=Rp)
    return cache[key]


def _make_geom(a, bid, mesh_assets=None, mesh_cache=None):
    gtype = a.get("type", "sphere")
    pos = np.array(_floats(a.get("pos", "0 0 0")))
    quat = qnorm(_floats(a.get("quat", "1 0 0 0")))
    contype = int(a.get("contype", 1))
    conaffinity = int(a.get("conaffinity", 1))
    surrogate = 0
    if gtype == "mesh" and mesh_assets is not None:
        cv = _load_convex(mesh_assets[a["mesh"]], mesh_cache)
        # the geom frame moves to the mesh's inertial frame (MuJoCo re-centres and re-aligns meshes)
        pos = pos + q2mat(quat) @ cv["com"]
        quat = qnorm(qmul(quat, mat2q(cv["R"])))
        hull = cv["hull"]
        size = list(np.max(np.abs(hull), axis=0))
        fr = _floats(a["friction"]) if "friction" in a else list(DEF_FRICTION)
        fr = (fr + list(DEF_FRICTION[len(fr):]))[:3]
        vol = cv["vol"]
        mass = float(a["mass"]) if "mass" in a else DENSITY * vol
        return dict(type=GEOM_MESH, body=bid, pos=pos, quat=quat, size=size, contype=contype,
                    conaffinity=conaffinity, condim=int(a.get("condim", 3)), priority=int(a.get("priority", 0)),
                    friction=fr, solref=_floats(a["solref"]) if "solref" in a else list(DEF_SOLREF),
                    solimp=_pad_solimp(_floats(a["solimp"])) if "solimp" in a else list(DEF_SOLIMP),
                    margin=float(a.get("margin", 0.0)), gap=float(a.get("gap", 0.0)),
                    solmix=float(a.get("solmix", 1.0)), mass=mass,
                    rbound=float(np.max(np.linalg.norm(hull, axis=1))), surrogate=0,
                    mesh=a["mesh"], hull=hull, inertia_diag=np.asarray(cv["inertia"]) * (mass / vol))
    if gtype == "mesh":
        half, center, collide = MESH_SURROGATE[a["mesh"]]
        pos = pos + q2mat(quat) @ np.array(center)
        size = list(half)
        t = GEOM_BOX
        surrogate = 1
        if not collide:
            contype = conaffinity = 0
    elif gtype == "box":
        size = _floats(a["size"])
        t = GEOM_BOX
    elif gtype == "plane":
        size = (_floats(a.get("size", "0 0 1")) + [0.0] * 3)[:3]
        t = GEOM_PLANE
    else:
        raise ValueError(f"unsupported geom type {gtype}")
    fr = _floats(a["friction"]) if "friction" in a else list(DEF_FRICTION)
    fr = (fr + list(DEF_FRICTION[len(fr):]))[:3]
    if t == GEOM_BOX:
        vol = 8.0 * size[0] * size[1] * size[2]
        rbound = math.sqrt(size[0] ** 2 + size[1] ** 2 + size[2] ** 2)
    else:
        vol = 0.0
        rbound = 0.0
    mass = float(a["mass"]) if "mass" in a else DENSITY * vol
    return dict(type=t, body=bid, pos=pos, quat=quat, size=size, contype=contype, conaffinity=conaffinity,
                condim=int(a.get("condim", 3)), priority=int(a.get("priority", 0)), friction=fr,
                solref=_floats(a["solref"]) if "solref" in a else list(DEF_SOLREF),
                solimp=_pad_solimp(_floats(a["solimp"])) if "solimp" in a else list(DEF_SOLIMP),
                margin=float(a.get("margin", 0.0)), gap=float(a.get("gap", 0.0)),
                solmix=float(a.get("solmix", 1.0)), mass=mass, rbound=rbound, surrogate=surrogate)


def _inertia_from_geoms(gs):
    """mjCBody inertiafromgeom: sum geom masses, com, composite inertia."""
    gs = [g for g in gs if g["type"] != GEOM_PLANE]
    mass = sum(g["mass"] for g in gs)
    if mass <= 0:
        return 0.0, np.zeros(3), np.array([1.0, 0, 0, 0]), np.zeros(3)
    com = sum(g["mass"] * g["pos"] for g in gs) / mass
    I = np.zeros((3, 3))
    for g in gs:
        a, b, c = g["size"]
        m = g["mass"]
        if g["type"] == GEOM_MESH:  # principal inertia of the mesh solid, in the geom (inertial) frame
            Ig = np.diag(g["inertia_diag"])
        else:
            Ig = np.diag([m / 3 * (b * b + c * c), m / 3 * (a * a + c * c), m / 3 * (a * a + b * b)])
        R = q2mat(g["quat"])
        d = g["pos"] - com
        I += R @ Ig @ R.T + m * (np.dot(d, d) * np.eye(3) - np.outer(d, d))
    off = abs(I[0, 1]) + abs(I[0, 2]) + abs(I[1, 2])
    if off < 1e-14 * max(1e-30, np.trace(I)):
        return mass, com, np.array([1.0, 0, 0, 0]), np.diag(I).copy()
    w, V = np.linalg.eigh(I)
    if np.linalg.det(V) < 0:
        V[:, 2] = -V[:, 2]
    return mass, com, mat2q(V), w


def _mix_params(g1, g2):
    """MuJoCo contact parameter mixing (mj_contactParam / mjCPair defaults)."""
    if g1["priority"] != g2["priority"]:
        src = g1 if g1["priority"] > g2["priority"] else g2
        condim = src["condim"]
        fr = list(src["friction"])
        solref = list(src["solref"])
        solimp = list(src["solimp"])
    else:
        condim = max(g1["condim"], g2["condim"])
        s1, s2 = g1["solmix"], g2["solmix"]
        if s1 < 1e-15 and s2 < 1e-15:
            mix = 0.5
        elif s1 < 1e-15:
            mix = 0.0
        elif s2 < 1e-15:
            mix = 1.0
        else:
            mix = s1 / (s1 + s2)
        fr = [max(g1["friction"][i], g2["friction"][i]) for i in range(3)]
        if g1["solref"][0] > 0 and g2["solref"][0] > 0:
            solref = [mix * g1["solref"][i] + (1 - mix) * g2["solref"][i] for i in range(2)]
        else:
            solref = [min(g1["solref"][i], g2["solref"][i]) for i in range(2)]
        solimp = [mix * g1["solimp"][i] + (1 - mix) * g2["solimp"][i] for i in range(5)]
    return dict(condim=condim, friction=[fr[0], fr[0], fr[1], fr[2], fr[2]], solref=solref, solimp=solimp,
                margin=max(g1["margin"], g2["margin"]), gap=max(g1["gap"], g2["gap"]))


# ---------------------------------------------------------------------------
# mj_setConst equivalents at qpos0 (plain numpy; compile-time only)
def _fk(m, qpos):
    nb = m["nbody"]
    xpos = np.zeros((nb, 3))
    xquat = np.zeros((nb, 4))
    xquat[0] = [1, 0, 0, 0]
    xanchor = np.zeros((m["njnt"], 3))
    xaxis = np.zeros((m["njnt"], 3))
    for i in range(1, nb):
        p = m["body_parentid"][i]
        bp = np.array(m["body_pos"][i])
        bq = np.array(m["body_quat"][i])
        if m["body_jntnum"][i] and m["jnt_type"][m["body_jntadr"][i]] == JNT_FREE:
            j = m["body_jntadr"][i]
            a = m["jnt_qposadr"][j]
            pos = qpos[a:a + 3].copy()
            quat = qnorm(qpos[a + 3:a + 7])
            xanchor[j] = pos
            xaxis[j] = [0, 0, 1]
        else:
            pos = xpos[p] + q2mat(xquat[p]) @ bp
            quat = qmul(xquat[p], bq)
            for k in range(m["body_jntnum"][i]):
                j = m["body_jntadr"][i] + k
                ax = np.array(m["jnt_axis"][j])
                R = q2mat(quat)
                xaxis[j] = R @ ax
                xanchor[j] = R @ np.array(m["jnt_pos"][j]) + pos
                ang = qpos[m["jnt_qposadr"][j]] - m["qpos0"][m["jnt_qposadr"][j]]
                ql = np.array([math.cos(ang / 2)] + list(math.sin(ang / 2) * ax))
                quat = qmul(quat, ql)
                pos = xanchor[j] - q2mat(quat) @ np.array(m["jnt_pos"][j])
        xpos[i] = pos
        xquat[i] = qnorm(quat)
    xmat = np.array([q2mat(q) for q in xquat])
    xipos = np.array([xpos[i] + xmat[i] @ np.array(m["body_ipos"][i]) for i in range(nb)])
    return xpos, xmat, xipos, xanchor, xaxis


def _mass_matrix(m, qpos):
    nb, nv = m["nbody"], m["nv"]
    xpos, xmat, xipos, xanchor, xaxis = _fk(m, qpos)
    mass = np.array(m["body_mass"])
    sub = np.zeros((nb, 3))
    for i in range(nb):
        sub[i] = mass[i] * xipos[i]
    for i in range(nb - 1, 0, -1):
        sub[m["body_parentid"][i]] += sub[i]
    stm = np.array(m["body_subtreemass"])
    subcom = np.array([sub[i] / stm[i] if stm[i] > 1e-15 else xipos[i] for i in range(nb)])
    # cdof (MuJoCo mj_comPos)
    cdof = np.zeros((nv, 6))
    for j in range(m["njnt"]):
        b = m["jnt_bodyid"][j]
        off = subcom[m["body_rootid"][b]] - xanchor[j]
        da = m["jnt_dofadr"][j]
        if m["jnt_type"][j] == JNT_FREE:
            for k in range(3):
                cdof[da + k, 3 + k] = 1.0
            for k in range(3):
                ax = xmat[b][:, k]
                cdof[da + 3 + k, :3] = ax
                cdof[da + 3 + k, 3:] = np.cross(ax, off)
        else:
            cdof[da, :3] = xaxis[j]
            cdof[da, 3:] = np.cross(xaxis[j], off)
    # spatial inertias about root subtree com, 6x6 [ang; lin]
    I6 = np.zeros((nb, 6, 6))
    for i in range(1, nb):
        R = xmat[i] @ q2mat(m["body_iquat"][i])
        Ic = R @ np.diag(m["body_inertia"][i]) @ R.T
        d = xipos[i] - subcom[m["body_rootid"][i]]
        dx = np.array([[0, -d[2], d[1]], [d[2], 0, -d[0]], [-d[1], d[0], 0]])
        mm = mass[i]
        I6[i, :3, :3] = Ic - mm * dx @ dx
        I6[i, :3, 3:] = mm * dx
        I6[i, 3:, :3] = -mm * dx
        I6[i, 3:, 3:] = mm * np.eye(3)
    crb = I6.copy()
    for i in range(nb - 1, 0, -1):
        p = m["body_parentid"][i]
        if p > 0:
            crb[p] += crb[i]
    M = np.zeros((nv, nv))
    for i in range(nv):
        buf = crb[m["dof_bodyid"][i]] @ cdof[i]
        j = i
        while j >= 0:
            M[i, j] += cdof[j] @ buf
            M[j, i] = M[i, j]
            j = m["dof_parentid"][j]
        M[i, i] += m["dof_armature"][i]
    return M, cdof, subcom, xpos, xmat, xipos


def _set_const(m):
    nv, nb = m["nv"], m["nbody"]
    qpos0 = np.array(m["qpos0"])
    M, cdof, subcom, xpos, xmat, xipos = _mass_matrix(m, qpos0)
    Minv = np.linalg.inv(M) if nv else np.zeros((0, 0))
    m["meaninertia"] = float(np.trace(M) / nv) if nv else 1.0
    inv0 = np.zeros((nb, 2))
    for i in range(1, nb):
        if m["body_weldid"][i] == 0:
            continue
        J = np.zeros((6, nv))
        # dofs in chain of body i
        d = -1
        k = i
        while k > 0 and d < 0:
            if m["body_dofnum"][k]:
                d = m["body_dofadr"][k] + m["body_dofnum"][k] - 1
            k = m["body_parentid"][k]
        off = xipos[i] - subcom[m["body_rootid"][i]]
        while d >= 0:
            J[0:3, d] = cdof[d, 3:] + np.cross(cdof[d, :3], off)
            J[3:6, d] = cdof[d, :3]
            d = m["dof_parentid"][d]
        A = J @ Minv @ J.T
        inv0[i, 0] = (A[0, 0] + A[1, 1] + A[2, 2]) / 3
        inv0[i, 1] = (A[3, 3] + A[4, 4] + A[5, 5]) / 3
    m["body_invweight0"] = inv0.tolist()
    dinv = np.zeros(nv)
    for j in range(m["njnt"]):
        da = m["jnt_dofadr"][j]
        if m["jnt_type"][j] == JNT_FREE:
            dinv[da:da + 3] = np.mean([Minv[da + k, da + k] for k in range(3)])
            dinv[da + 3:da + 6] = np.mean([Minv[da + 3 + k, da + 3 + k] for k in range(3)])
        else:
            dinv[da] = Minv[da, da]
    m["dof_invweight0"] = dinv.tolist()
    # connect anchors in body2 frame at qpos0
    for e in range(m["neq"]):
        if m["eq_type"][e] == EQ_CONNECT:
            b1, b2 = m["eq_obj1"][e], m["eq_obj2"][e]
            a1 = np.array(m["eq_data"][e][0:3])
            pw = xpos[b1] + xmat[b1] @ a1
            a2 = xmat[b2].T @ (pw - xpos[b2])
            m["eq_data"][e][3:6] = a2.tolist()


# ---------------------------------------------------------------------------
# C struct mirror of include/ur3e_model.h
_d = ctypes.c_double
_i = ctypes.c_int


class UR3eModelC(ctypes.Structure):
    _fields_ = [
        ("version", _i),
        ("nq", _i), ("nv", _i), ("nu", _i), ("nbody", _i), ("njnt", _i), ("ngeom", _i), ("nsite", _i),
        ("ncpair", _i), ("neq", _i), ("ntendon", _i), ("nkey", _i), ("ntouch", _i),
        ("timestep", _d), ("gravity", _d * 3), ("cone", _i), ("impratio", _d), ("tolerance", _d),
        ("iterations", _i), ("ls_iterations", _i), ("ls_tolerance", _d), ("meaninertia", _d),
        ("body_parentid", _i * MAXBODY), ("body_rootid", _i * MAXBODY), ("body_weldid", _i * MAXBODY),
        ("body_jntnum", _i * MAXBODY), ("body_jntadr", _i * MAXBODY), ("body_dofnum", _i * MAXBODY),
        ("body_dofadr", _i * MAXBODY),
        ("body_pos", (_d * 3) * MAXBODY), ("body_quat", (_d * 4) * MAXBODY), ("body_ipos", (_d * 3) * MAXBODY),
        ("body_iquat", (_d * 4) * MAXBODY), ("body_mass", _d * MAXBODY), ("body_subtreemass", _d * MAXBODY),
        ("body_inertia", (_d * 3) * MAXBODY), ("body_invweight0", (_d * 2) * MAXBODY),
        ("jnt_type", _i * MAXJNT), ("jnt_qposadr", _i * MAXJNT), ("jnt_dofadr", _i * MAXJNT),
        ("jnt_bodyid", _i * MAXJNT), ("jnt_limited", _i * MAXJNT),
        ("jnt_pos", (_d * 3) * MAXJNT), ("jnt_axis", (_d * 3) * MAXJNT), ("jnt_range", (_d * 2) * MAXJNT),
        ("jnt_stiffness", _d * MAXJNT), ("jnt_margin", _d * MAXJNT), ("jnt_solref", (_d * 2) * MAXJNT),
        ("jnt_solimp", (_d * 5) * MAXJNT),
        ("dof_bodyid", _i * MAXNV), ("dof_jntid", _i * MAXNV), ("dof_parentid", _i * MAXNV),
        ("dof_armature", _d * MAXNV), ("dof_damping", _d * MAXNV), ("dof_frictionloss", _d * MAXNV),
        ("dof_invweight0", _d * MAXNV), ("dof_solref", (_d * 2) * MAXNV), ("dof_solimp", (_d * 5) * MAXNV),
        ("qpos0", _d * MAXNQ), ("qpos_spring", _d * MAXNQ),
        ("geom_type", _i * MAXGEOM), ("geom_bodyid", _i * MAXGEOM), ("geom_surrogate", _i * MAXGEOM),
        ("geom_pos", (_d * 3) * MAXGEOM), ("geom_quat", (_d * 4) * MAXGEOM), ("geom_size", (_d * 3) * MAXGEOM),
        ("geom_rbound", _d * MAXGEOM),
        ("site_bodyid", _i * MAXSITE), ("site_type", _i * MAXSITE), ("site_pos", (_d * 3) * MAXSITE),
        ("site_quat", (_d * 4) * MAXSITE), ("site_size", (_d * 3) * MAXSITE),
        ("cpair_geom1", _i * MAXCPAIR), ("cpair_geom2", _i * MAXCPAIR), ("cpair_explicit", _i * MAXCPAIR),
        ("cpair_condim", _i * MAXCPAIR), ("cpair_friction", (_d * 5) * MAXCPAIR),
        ("cpair_solref", (_d * 2) * MAXCPAIR), ("cpair_solimp", (_d * 5) * MAXCPAIR),
        ("cpair_margin", _d * MAXCPAIR), ("cpair_gap", _d * MAXCPAIR),
        ("ten_num", _i * MAXTEN), ("ten_dof", (_i * MAXTENWRAP) * MAXTEN), ("ten_coef", (_d * MAXTENWRAP) * MAXTEN),
        ("eq_type", _i * MAXEQ), ("eq_obj1", _i * MAXEQ), ("eq_obj2", _i * MAXEQ),
        ("eq_data", (_d * 11) * MAXEQ), ("eq_solref", (_d * 2) * MAXEQ), ("eq_solimp", (_d * 5) * MAXEQ),
        ("act_trntype", _i * MAXU), ("act_trnid", _i * MAXU), ("act_gaintype", _i * MAXU),
        ("act_biastype", _i * MAXU), ("act_ctrllimited", _i * MAXU), ("act_forcelimited", _i * MAXU),
        ("act_ctrlrange", (_d * 2) * MAXU), ("act_forcerange", (_d * 2) * MAXU),
        ("act_gainprm", (_d * 3) * MAXU), ("act_biasprm", (_d * 3) * MAXU), ("act_gear", _d * MAXU),
        ("touch_site", _i * MAXTOUCH),
        ("key_qpos", (_d * MAXNQ) * MAXKEY), ("key_qvel", (_d * MAXNV) * MAXKEY),
        ("id_site_tcp", _i), ("id_site_handle", _i), ("id_site_lpad", _i), ("id_site_rpad", _i),
        ("id_body_fish", _i), ("id_body_ghost", _i), ("id_body_lpad", _i), ("id_body_rpad", _i),
        ("id_key_home", _i), ("id_key_down", _i),
        ("mask_arm_bodies", ctypes.c_uint), ("mask_gripper_bodies", ctypes.c_uint),
        ("fish_topple_z", _d),
        ("id_body_table", _i),
        ("fish_half_z", _d),
        ("nsensor", _i), ("nsensordata", _i), ("sensor_type", _i * MAXSENSOR), ("sensor_objid", _i * MAXSENSOR),
        ("sensor_adr", _i * MAXSENSOR),
        ("nmesh", _i), ("nmeshvert", _i), ("geom_dataid", _i * MAXGEOM), ("mesh_vertadr", _i * MAXMESH),
        ("mesh_vertnum", _i * MAXMESH), ("mesh_vert", (_d * 3) * MAXMESHVERT),
    ]


# fields a model dict may omit (images compiled before mesh support: no mesh geoms)
_OPTIONAL_ZERO = {"nmesh", "nmeshvert", "geom_dataid", "mesh_vertadr", "mesh_vertnum", "mesh_vert"}


def _fill(dst, val):
    """Recursively copy nested lists into a ctypes array."""
    if isinstance(val, (list, tuple, np.ndarray)):
        for i, v in enumerate(val):
            if isinstance(v, (list, tuple, np.ndarray)):
                _fill(dst[i], v)
            else:
                dst[i] = v
    else:
        raise TypeError


def to_ctypes(m: dict) -> UR3eModelC:
    c = UR3eModelC()
    for name, _t in UR3eModelC._fields_:
        if name not in m:
            if name in _OPTIONAL_ZERO:
                continue
            raise KeyError(f"model dict lacks {name}")
        v = m[name]
        if isinstance(v, (list, tuple, np.ndarray)):
            _fill(getattr(c, name), v)
        else:
            setattr(c, name, v)
    return c


def save_json(m: dict, path: str) -> None:
    with open(path, "w") as f:
        json.dump(m, f, indent=1, sort_keys=True)


def load_json(path: str) -> dict:
    with open(path) as f:
        return json.load(f)
