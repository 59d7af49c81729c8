"""The C ABI's MJCF / YAML entry points (include/ur3e_batch.h: ur3e_model_from_mjcf,
ur3e_config_gains_from_yaml; ur3e_amd/csrc/ur3e_mjcf.cpp) called by a program that is not Python
(tests/c/mjcf_driver.c, built here with gcc) and in-process through ctypes (the running interpreter's
branch).  No GPU: the model image and the gains are compared byte for byte with the Python compiler's
(ur3e_amd/model/compiler.py) and the YAML reader's (ur3e_amd/gains.py) own results; with the reference
checkout present, its assets/main.xml compiles through the ABI to the committed model image."""
import ctypes
import os
import struct
import subprocess

import numpy as np
import pytest
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASSETS = os.path.join(ROOT, "tests", "assets")
LIBDIR = os.path.join(ROOT, "ur3e_amd", "_lib")
REF_MAIN = "/root/reference/assets/main.xml"


def build_driver(out_dir):
    exe = os.path.join(str(out_dir), "mjcf_driver")
    subprocess.run(["gcc", "-O1", "-D__HIP_PLATFORM_AMD__", "-I", os.path.join(ROOT, "include"), "-I",
                    "/opt/rocm/include", os.path.join(ROOT, "tests", "c", "mjcf_driver.c"), "-o", exe,
                    "-L", LIBDIR, "-lur3e_amd", f"-Wl,-rpath,{LIBDIR}", "-L", "/opt/rocm/lib", "-lamdhip64",
                    "-Wl,-rpath,/opt/rocm/lib"], check=True)
    return exe


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    if not os.path.exists(os.path.join(LIBDIR, "libur3e_amd.so")):
        pytest.skip("library not built")
    return build_driver(tmp_path_factory.mktemp("drv"))


def _run(args, **kw):
    env = dict(os.environ)
    env.pop("PYTHONPATH", None)  # the library finds the package beside itself
    return subprocess.run(args, capture_output=True, text=True, timeout=300, env=env, **kw)


@pytest.mark.parametrize("xml", ["kat_box_plane.xml", "mesh_scene.xml", "kat_connect.xml"])
def test_c_caller_compiles_mjcf_to_the_python_image(driver, tmp_path, xml):
    from ur3e_amd.model.compiler import compile_mjcf, to_ctypes
    out = tmp_path / "m.bin"
    r = _run([driver, "image", os.path.join(ASSETS, xml), str(out)], cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr
    assert out.read_bytes() == bytes(to_ctypes(compile_mjcf(os.path.join(ASSETS, xml))))


@pytest.mark.skipif(not os.path.exists(REF_MAIN), reason="reference checkout absent (GPU box)")
def test_c_caller_compiles_reference_main_xml(driver, tmp_path):
    """assets/main.xml of the reference, through the ABI, is the committed model image (its meshes are
    absent, so the box surrogate: compile_mjcf's 'auto')."""
    from ur3e_amd import runtime as rt
    out = tmp_path / "main.bin"
    r = _run([driver, "image", REF_MAIN, str(out)], cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr
    assert "nq=21 nv=20 nu=7" in r.stdout
    assert out.read_bytes() == bytes(rt.load_model("main")[1])


def test_c_caller_gains_from_yaml(driver, tmp_path):
    from ur3e_amd import gains, runtime as rt
    out = tmp_path / "g.bin"
    # defaults (no path, no controller/config under the cwd): the packaged copies of the reference's files
    r = _run([driver, "gains", "-", str(rt.TASK_GYM_V2), str(out)], cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr
    g = struct.unpack("<36d", out.read_bytes())
    tg = gains.task_gains()
    assert list(g[:12]) == tg["kp_pos"] + tg["kd_pos"] + tg["kp_rot"] + tg["kd_rot"]
    # an explicit move_j file (move_j.py:46-52 reads config_j.yml)
    p = tmp_path / "j.yml"
    p.write_text(yaml.safe_dump(dict(hold=10, qpos=dict(kp=[1.0, 2, 3, 4, 5, 6], kd=[7.0, 8, 9, 10, 11, 12])), sort_keys=False))
    r = _run([driver, "gains", str(p), str(rt.TASK_MOVE_J), str(out)], cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr
    g = struct.unpack("<36d", out.read_bytes())
    assert list(g[12:24]) == [1.0, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12]
    # a malformed file fails with the reader's error, not a crash
    p.write_text(yaml.safe_dump(dict(hold=10, qpos=dict(kp=[1.0] * 5, kd=[1.0] * 6)), sort_keys=False))
    r = _run([driver, "gains", str(p), str(rt.TASK_MOVE_J), str(out)], cwd=str(tmp_path))
    assert r.returncode == 1 and "expected 6 gains" in r.stderr


def test_missing_mjcf_is_an_error(driver, tmp_path):
    r = _run([driver, "image", str(tmp_path / "nope.xml"), str(tmp_path / "m.bin")])
    assert r.returncode == 1 and "no such MJCF file" in r.stderr
    r = _run([driver, "image", os.path.join(ASSETS, "missing_mesh.xml"), str(tmp_path / "m.bin")])
    assert r.returncode == 1 and "ur3e_model_from_mjcf" in r.stderr


def test_missing_libpython_is_an_error_code(driver, tmp_path):
    """UR3E_LIBPYTHON naming a library that does not exist (a C host without an interpreter linked in): the
    entry point returns UR3E_EINVAL with the loader's message -- no crash out of the extern "C" call."""
    env = dict(os.environ)
    env.pop("PYTHONPATH", None)
    env["UR3E_LIBPYTHON"] = str(tmp_path / "no_such_libpython.so")
    r = subprocess.run([driver, "image", os.path.join(ASSETS, "kat_box_plane.xml"), str(tmp_path / "m.bin")],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 1, (r.returncode, r.stderr)
    assert "libpython not found" in r.stderr and "no_such_libpython.so" in r.stderr


def test_non_ascii_paths(driver, tmp_path):
    """An MJCF (and its mesh files) under a directory whose name is not ASCII, and an output path there: the
    embedded compiler receives the same bytes (a bytes literal decoded with the filesystem encoding)."""
    import shutil
    from ur3e_amd.model.compiler import compile_mjcf, to_ctypes
    d = tmp_path / "modèle_ä"
    shutil.copytree(ASSETS, d)
    out = d / "sortie_é.bin"
    r = _run([driver, "image", str(d / "mesh_scene.xml"), str(out)], cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr
    assert out.read_bytes() == bytes(to_ctypes(compile_mjcf(os.path.join(ASSETS, "mesh_scene.xml"))))


def test_in_process_ctypes_uses_the_running_interpreter():
    from ur3e_amd import runtime as rt
    from ur3e_amd.model.compiler import compile_mjcf, to_ctypes
    L = rt.load_library()
    L.ur3e_model_from_mjcf.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_void_p]
    ref = to_ctypes(compile_mjcf(os.path.join(ASSETS, "mesh_scene.xml")))
    out = type(ref)()
    rc = L.ur3e_model_from_mjcf(os.path.join(ASSETS, "mesh_scene.xml").encode(), b"auto", ctypes.byref(out))
    assert rc == 0, L.ur3e_last_error()
    assert bytes(out) == bytes(ref)
    assert np.frombuffer(bytes(out), np.uint8).any()
