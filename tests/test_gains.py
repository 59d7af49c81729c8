"""Controller gains from the YAML configs (ur3e_amd/gains.py), the way the reference reads them:
positional unpacking of each section (controller_func.py:90-91, :136), cwd-relative
controller/config/<name> (ur3e_env2.py:66), an explicit path overriding both (CPU only)."""
import os

import numpy as np
import pytest
import yaml

from ur3e_amd import gains
from ur3e_amd import runtime as rt

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_packaged_configs_equal_reference_values():
    assert gains.task_gains() == rt.GAINS_L_MUG
    assert gains.joint_gains() == rt.GAINS_J
    pos, rot = gains.move_l_gains()
    assert pos == rt.GAINS_L_POS and rot == rt.GAINS_L_ROT
    assert gains.hold() == 120 and gains.hold("config_j.yml") == 120 and gains.hold("config_l.yml") == 120


def test_reference_golden_gains():
    g = np.load(os.path.join(GOLDEN, "reference_golden.npz"))
    pos, rot = gains.move_l_gains()
    np.testing.assert_array_equal([pos["kp"], pos["kd"]], g["cfgl_pos"])
    np.testing.assert_array_equal([rot["kp"], rot["kd"]], g["cfgl_rot"])


def _write(path, d):
    with open(path, "w") as f:
        yaml.safe_dump(d, f, sort_keys=False)


def test_positional_unpacking_and_cwd(tmp_path, monkeypatch):
    d = dict(hold=60, pos=dict(kp=[1.0, 2.0, 3.0], kd=[4.0, 5.0, 6.0], ki=[0, 0, 0]),
             rot=dict(kd=[7.0, 8.0, 9.0], kp=[10.0, 11.0, 12.0], ki=[0, 0, 0]))  # rot: kd written first
    os.makedirs(tmp_path / "controller" / "config")
    _write(tmp_path / "controller" / "config" / "config_l_mug.yml", d)
    monkeypatch.chdir(tmp_path)
    g = gains.task_gains()
    # file order decides: the first entry is kp whatever its name (controller_func.py:90-91)
    assert g == dict(kp_pos=[1.0, 2.0, 3.0], kd_pos=[4.0, 5.0, 6.0], kp_rot=[7.0, 8.0, 9.0], kd_rot=[10.0, 11.0, 12.0])
    assert gains.hold() == 60
    # an explicit path wins over the working directory
    p = tmp_path / "other.yml"
    d["pos"]["kp"] = [100.0, 200.0, 300.0]
    _write(p, d)
    assert gains.task_gains(str(p))["kp_pos"] == [100.0, 200.0, 300.0]
    # the spec of a config_l_mug env picks the file up at construction; v0 keeps its hard-coded gains
    from ur3e_amd.envs.specs import spec
    assert spec("gymnasium_env/ur3e-v2")["gains"]["kp_pos"] == [1.0, 2.0, 3.0]
    assert spec("gymnasium_env/ur3e-v2", str(p))["gains"]["kp_pos"] == [100.0, 200.0, 300.0]
    assert spec("gymnasium_env/ur3e-v0")["gains"] == rt.GAINS_V0


def test_malformed_sections_raise(tmp_path):
    p = tmp_path / "bad.yml"
    _write(p, dict(hold=120, pos=dict(kp=[1.0, 2.0, 3.0], kd=[4.0, 5.0, 6.0]), rot=dict(kp=[1, 2, 3], kd=[1, 2, 3], ki=[0, 0, 0])))
    with pytest.raises(ValueError):  # two entries where the reference unpacks three
        gains.task_gains(str(p))
    _write(p, dict(hold=120, qpos=dict(kp=[1.0] * 5, kd=[1.0] * 6)))
    with pytest.raises(ValueError):
        gains.joint_gains(str(p))
    with pytest.raises(FileNotFoundError):
        gains.task_gains(str(tmp_path / "missing.yml"))


def test_make_config_reads_move_j_move_l_yaml(tmp_path):
    """move_j / move_l configs take their pd_joint_ctrl gains from config_j.yml / config_l.yml
    (move_j.py:46-52, move_l.py:92-99) when none are given, and from an explicit path when one is."""
    cj = rt.make_config(task=rt.TASK_MOVE_J)
    assert list(cj.joint_gains) == gains.joint_gains()["kp"] + gains.joint_gains()["kd"]
    p = tmp_path / "j.yml"
    _write(p, dict(hold=100, qpos=dict(kp=[1.0, 2.0, 3.0, 4.0, 5.0, 6.0], kd=[0.5] * 6)))
    cj = rt.make_config(task=rt.TASK_MOVE_J, config_yaml_path=str(p))
    assert list(cj.joint_gains) == [1.0, 2.0, 3.0, 4.0, 5.0, 6.0] + [0.5] * 6
    p = tmp_path / "l.yml"
    _write(p, dict(hold=100, pos=dict(kp=[7.0] * 6, kd=[8.0] * 6), rot=dict(kp=[9.0] * 6, kd=[10.0] * 6)))
    cl = rt.make_config(task=rt.TASK_MOVE_L, config_yaml_path=str(p))
    assert list(cl.joint_gains) == [7.0] * 6 + [8.0] * 6
    assert list(cl.rot_joint_gains) == [9.0] * 6 + [10.0] * 6
    # explicit gains still win
    cl = rt.make_config(task=rt.TASK_MOVE_L, joint_gains=dict(kp=[1.0] * 6, kd=[2.0] * 6), config_yaml_path=str(p))
    assert list(cl.joint_gains) == [1.0] * 6 + [2.0] * 6 and list(cl.rot_joint_gains) == [9.0] * 6 + [10.0] * 6


def test_output_buffers_checked_before_launch():
    """Batch.out_ptr (used by get_actuator_force(out) and task_space_state(batch, out)) rejects a buffer
    the kernel would write out of bounds: wrong dtype, shape, device or a non-contiguous view."""
    import types

    import torch
    fake = types.SimpleNamespace(torch=torch, device=torch.device("cpu"), n=4)
    ok = torch.zeros((4, 7), dtype=torch.float64)
    assert rt.Batch.out_ptr(fake, ok, 7, "t").value == ok.data_ptr()
    rec = torch.zeros((3, 4, 7), dtype=torch.float64)
    assert rt.Batch.out_ptr(fake, rec[1], 7, "t").value == rec[1].data_ptr()  # a row of a recording buffer
    for bad in (torch.zeros((4, 7), dtype=torch.float32), torch.zeros((4, 6), dtype=torch.float64),
                torch.zeros((3, 7), dtype=torch.float64), torch.zeros((7, 4), dtype=torch.float64).t(),
                torch.zeros((4, 7), dtype=torch.float64, device="meta"), ok.numpy()):
        with pytest.raises(ValueError):
            rt.Batch.out_ptr(fake, bad, 7, "t")
