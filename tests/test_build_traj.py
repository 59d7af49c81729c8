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


def test_traj_l_golden(golden):
    hold = int(golden["trajl_hold"])
    for i in range(len(golden["trajl_start"])):
        tr = bt.build_traj_l(golden["trajl_start"][i], hold)
        assert tr.shape == (500 * hold, 7)
        np.testing.assert_array_equal(tr[::hold], golden["trajl_rows"][i])


def test_move_l_gains_match_config_l(golden):
    """runtime.GAINS_L_POS / GAINS_L_ROT are controller/config/config_l.yml's "pos" / "rot" PD gains."""
    from ur3e_amd import runtime as rt
    np.testing.assert_array_equal([rt.GAINS_L_POS["kp"], rt.GAINS_L_POS["kd"]], golden["cfgl_pos"])
    np.testing.assert_array_equal([rt.GAINS_L_ROT["kp"], rt.GAINS_L_ROT["kd"]], golden["cfgl_rot"])


def test_pick_place_torch_rows(golden):
    s = torch.from_numpy(golden["pp_start"])
    picks = torch.from_numpy(golden["pp_dest"][:, 0])
    places = torch.from_numpy(golden["pp_dest"][:, 1])
    pp = bt.PickPlaceTorch(s, picks, places)
    for t in list(range(0, 7200, 97)) + [7199]:
        np.testing.assert_array_equal(pp.row(t).numpy(), golden["pp_rows"][:, t // 120])


def _aug_noise(seed, n=1):
    # np.random.seed(seed) + the reference's rand(rows, 7) calls == one RandomState stream in C order
    return np.random.RandomState(seed).random_sample((n, bt.AUG_NOISE_ROWS, 7))


def test_augmented_golden(golden):
    """build_traj_l_pick_place_imitation_augmented (build_traj.py:61-125) with np.random seeded."""
    idx = golden["aug_idx"]
    for i in range(len(golden["aug_start"])):
        rs = np.random.RandomState(int(golden["aug_seed"][i]))
        block, target = golden["aug_dest"][i]
        tr = bt.build_traj_l_pick_place_imitation_augmented(golden["aug_start"][i], [block, target], 120,
                                                            rand=rs.rand)
        assert tr.shape == (bt.AUG_T, 7)
        np.testing.assert_array_equal(tr[idx], golden["aug_rows"][i])


def test_augmented_torch_batch(golden):
    """The batched builder reproduces every golden trajectory from the same uniform stream."""
    idx = golden["aug_idx"]
    n = len(golden["aug_start"])
    noise = np.concatenate([_aug_noise(int(s)) for s in golden["aug_seed"]])
    aug = bt.AugmentedPickPlaceTorch(torch.from_numpy(golden["aug_start"]), torch.from_numpy(golden["aug_dest"][:, 0]),
                                     torch.from_numpy(golden["aug_dest"][:, 1]), torch.from_numpy(noise))
    assert aug.traj.shape == (bt.AUG_T, n, 7)
    for i in range(n):
        np.testing.assert_array_equal(aug.traj[:, i].numpy()[idx], golden["aug_rows"][i])
