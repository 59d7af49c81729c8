"""Host logic of the batched demo collector (controller/collect_demos.py): frame stacking
(collect_demos.py:21-57, restated here with the reference's deque algorithm) and the pickle
round trip of save_demos (:192-211).  GPU parity of the collection loop is in test_gpu_parity.py."""
from collections import deque

import numpy as np

from ur3e_amd.controller.collect_demos import Trajectory, save_demos, stack_expert_trajectories


def _deque_stack(obs, h):
    hist, out = deque(maxlen=h), []
    for i, o in enumerate(obs):
        if i == 0:
            for _ in range(h):
                hist.append(o)
        else:
            hist.append(o)
        out.append(np.array(hist))
    return np.array(out)


def test_stack_matches_deque():
    rng = np.random.default_rng(0)
    trajs = [Trajectory(obs=rng.normal(size=(n + 1, 24)), acts=rng.normal(size=(n, 4)),
                        infos=np.array([{}] * n), terminal=True) for n in (1, 5, 40)]
    for h in (1, 3, 8):
        out = stack_expert_trajectories(trajs, h)
        for a, b in zip(trajs, out):
            np.testing.assert_array_equal(b.obs, _deque_stack(a.obs, h))
            assert b.acts is a.acts and b.terminal


def test_save_demos_appends(tmp_path):
    p = str(tmp_path / "demos" / "expert_demos_indirect.pkl")
    t = [Trajectory(obs=np.zeros((3, 24)), acts=np.zeros((2, 4)), infos=None, terminal=True)]
    assert save_demos(t, p) == 1
    assert save_demos(t + t, p, resume_collecting=True) == 3
    assert save_demos(t, p, resume_collecting=False) == 1
