"""Trajectory builders vs golden rows from controller/build_traj.py."""
import numpy as np
import torch

from ur3e_amd.controller import build_traj as bt


def test_pick_place_golden(golden):
    for i in range(len(golden["pp_start"])):
        s = golden["pp_start"][i]
        pick, place = golden["pp_dest"][i]
        tr = bt.build_traj_l_pick_place(s, [pick, place], 120)
        assert tr.shape[0] == golden["pp_T"][i] == 7200
        np.testing.assert_array_equal(tr[::120], golden["pp_rows"][i])


def test_traj_j_golden(golden):
    for i in range(len(golden["trajj_start"])):
        tr = bt.build_traj_j(golden["trajj_start"][i], 120)
        assert tr.shape == (60000, 7)
        np.testing.assert_array_equal(tr[::120], golden["trajj_rows"][i])


def test_pick_place_torch_rows(golden):
    s = torch.from_numpy(golden["pp_start"])
    picks = torch.from_numpy(golden["pp_dest"][:, 0])
    places = torch.from_numpy(golden["pp_dest"][:, 1])
    pp = bt.PickPlaceTorch(s, picks, places)
    for t in list(range(0, 7200, 97)) + [7199]:
        np.testing.assert_array_equal(pp.row(t).numpy(), golden["pp_rows"][:, t // 120])
