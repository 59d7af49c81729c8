"""Trajectory builders (host side), restating controller/build_traj.py.

* build_traj_l_point_custom  (build_traj.py:215-254): 15-point linear segment
  (t[1:] of linspace(0, 1, 16)), each row held `hold` times.
* build_traj_l_pick_place    (build_traj.py:28-59): pick / up (+0.15 z, grip
  1 - g) / place (+0.025 z) / drop (grip 0); hold is hard-coded 120 (quirk:
  the `hold` argument is ignored).  Unlike the
  reference, `destinations` are not mutated in place.
* build_traj_j               (build_traj.py:387-470): np.random.seed(42) control
  points + cubic interp1d, 500 samples, held `hold` times, grip 0.
* build_traj_l               (build_traj.py:310-384): np.random.seed(49) task-space
  control points + cubic interp1d for x, y, z (the rotation draws are made and
  then overwritten with the fixed rotvec (-1.209, -1.209, 1.209)), grip 1, 500
  samples held `hold` times -- the move_l.main trajectory (controller/move_l.py:103).
* build_traj_l_pick_place_imitation_augmented (build_traj.py:61-125): seven
  15-point segments held 100 rows each (pick at start height / down / grab /
  up +0.15 / place / descend +0.025 / drop), uniform noise u/40 or u/20 on all
  but the last 500 rows of each segment (all rows of `up`); each segment starts
  from the previous segment's last (noisy) row.  `AugmentedPickPlaceTorch` is
  the batched GPU version used by controller/collect_demos.py.

Also a torch version of pick_place that evaluates rows analytically per env
and step on the GPU (`PickPlaceTorch`), used by the batched scripted driver
(controller/move_l_mug.py:67-81 semantics) without materialising [7200, 7]
per env.  Pinned against the reference by tests/golden (bit-exact).
"""
from __future__ import annotations

import numpy as np

HOLD_PICK_PLACE = 120
NUM_POINTS = 15


def _linear_rows(start, stop, num_points=NUM_POINTS):
    """scipy interp1d(kind='linear') on t_control=[0, 1] at linspace(0,1,n+1)[1:].

    scipy 1.15 routes 1-D linear interp1d to np.interp: slope*(x - x0) + y0,
    and x == x[-1] returns y[-1] exactly (so each segment ends exactly on `stop`)."""
    t = np.linspace(0, 1, num_points + 1)[1:]
    start = np.asarray(start, dtype=np.float64)
    stop = np.asarray(stop, dtype=np.float64)
    slope = (stop - start) / (1.0 - 0.0)
    rows = slope[None, :] * (t[:, None] - 0.0) + start[None, :]
    rows[-1] = stop
    return rows


def build_traj_l_point_custom(start, stop, hold, num_points=NUM_POINTS):
    return np.repeat(_linear_rows(start, stop, num_points), repeats=hold, axis=0)


def pick_place_waypoints(start, pick, place):
    """The 4 segment endpoint pairs (A, B) of build_traj_l_pick_place."""
    start = np.asarray(start, dtype=np.float64)
    pick = np.asarray(pick, dtype=np.float64)
    place = np.asarray(place, dtype=np.float64) + np.array([0, 0, 0.025, 0, 0, 0, 0])
    end_pick = _linear_rows(start, pick)[-1]
    up = end_pick + np.array([0, 0, 0.15, 0, 0, 0, 1 - end_pick[-1]])
    end_up = _linear_rows(end_pick, up)[-1]
    end_place = _linear_rows(end_up, place)[-1]
    drop = np.append(end_place[:-1], 0.0)
    return [(start, pick), (end_pick, up), (end_up, place), (end_place, drop)]


def build_traj_l_pick_place(start, destinations, hold=HOLD_PICK_PLACE):
    pick, place = destinations
    segs = pick_place_waypoints(start, pick, place)
    return np.vstack([build_traj_l_point_custom(a, b, HOLD_PICK_PLACE) for a, b in segs])


def build_traj_j(start, hold):
    from scipy.interpolate import interp1d
    num_points = 500
    t = np.linspace(0, 1, num_points)
    rs = np.random.RandomState(42)  # same MT19937 stream as np.random.seed(42)
    bounds = [[0.2, 0.5], [-0.3, 0.3], [0.4, 0.8], [0.4, 0.8], [0.4, 0.8], [0.4, 0.8]]
    ncp = 10
    t_control = np.linspace(0, 1, ncp + 1)
    cols = []
    for j in range(6):
        ctrl = np.concatenate([np.asarray(start, dtype=np.float64)[j:j + 1],
                               rs.uniform(bounds[j][0], bounds[j][1], ncp)])
        cols.append(interp1d(t_control, ctrl, kind="cubic")(t))
    g = np.tile([0, 0, 0], num_points // 3 + 1)[:num_points]
    return np.repeat(np.vstack(cols + [g]).T, repeats=hold, axis=0)


def build_traj_l(start, hold):
    from scipy.interpolate import interp1d
    num_points = 500
    t = np.linspace(0, 1, num_points)
    rs = np.random.RandomState(49)  # same MT19937 stream as np.random.seed(49)
    bounds = [[0.2, 0.5], [-0.3, 0.3], [0.4, 0.8], [-0.1, 0.1], [-0.1, 0.1], [-np.pi / 4, np.pi / 4]]
    ncp = 10
    t_control = np.linspace(0, 1, ncp + 1)
    start = np.asarray(start, dtype=np.float64)
    # all six control-point draws happen (in x, y, z, rx, ry, rz order) before the rotation columns are
    # replaced by constants, so the MT19937 stream advances exactly as in the reference
    ctrl = [np.concatenate([start[j:j + 1], rs.uniform(bounds[j][0], bounds[j][1], ncp)]) for j in range(6)]
    cols = [interp1d(t_control, ctrl[j], kind="cubic")(t) for j in range(3)]
    cols += [np.full(num_points, -1.209), np.full(num_points, -1.209), np.full(num_points, 1.209)]
    g = np.tile([1, 1, 1], num_points // 3 + 1)[:num_points]
    return np.repeat(np.vstack(cols + [g]).T, repeats=hold, axis=0)


# build_traj.py:70-73: noise norms; 500-row noiseless buffer at the end of each segment
AUG_HOLD = 100
AUG_BUFFER = 500
AUG_SEG_ROWS = NUM_POINTS * AUG_HOLD                       # 1500
AUG_T = 7 * AUG_SEG_ROWS                                    # 10500
# (noise norm, rows with noise) per segment: pick, down, grab, up, place, descend, drop
AUG_NOISE = [(40, AUG_SEG_ROWS - AUG_BUFFER), (40, AUG_SEG_ROWS - AUG_BUFFER), (20, AUG_SEG_ROWS - AUG_BUFFER),
             (20, AUG_SEG_ROWS), (20, AUG_SEG_ROWS - AUG_BUFFER), (20, AUG_SEG_ROWS - AUG_BUFFER),
             (20, AUG_SEG_ROWS - AUG_BUFFER)]
AUG_NOISE_ROWS = sum(r for _, r in AUG_NOISE)              # 7500 uniform rows of 7 per trajectory


def build_traj_l_pick_place_imitation_augmented(start, destinations, hold=None, rand=None):
    """build_traj.py:61-125 (`hold` is ignored there too: every segment holds 100 rows).

    rand(rows, 7) supplies the uniform noise in the reference's draw order (default: the global
    np.random.rand, as the reference)."""
    rand = np.random.rand if rand is None else rand
    block, target = (np.asarray(x, dtype=np.float64) for x in destinations)
    start = np.asarray(start, dtype=np.float64)

    def seg(a, b, k):
        norm, nrows = AUG_NOISE[k]
        tr = build_traj_l_point_custom(a, b, AUG_HOLD)
        noise = rand(nrows, 7) / norm
        if nrows < tr.shape[0]:
            noise = np.vstack([noise, np.zeros((tr.shape[0] - nrows, 7))])
        return tr + noise

    pick = np.hstack([block[:2], [start[2]], block[3:]])
    t_pick = seg(start, pick, 0)
    down = np.hstack([t_pick[-1, :2], [block[2]], t_pick[-1, 3:]])
    t_down = seg(t_pick[-1, :], down, 1)
    grab = np.append(t_down[-1, :-1], 1)
    t_grab = seg(t_down[-1, :], grab, 2)
    up = t_grab[-1, :] + [0, 0, 0.15, 0, 0, 0, 0]
    t_up = seg(t_grab[-1, :], up, 3)
    place = np.hstack([target[:2], t_up[-1, 2], target[3:]])
    t_place = seg(t_up[-1, :], place, 4)
    descend = target + [0, 0, 0.025, 0, 0, 0, 0]
    t_descend = seg(t_place[-1, :], descend, 5)
    end_drop = np.append(t_descend[-1, :-1], 0)
    t_drop = seg(t_descend[-1, :], end_drop, 6)
    return np.vstack([t_pick, t_down, t_grab, t_up, t_place, t_descend, t_drop])


class AugmentedPickPlaceTorch:
    """build_traj_l_pick_place_imitation_augmented for N trajectories at once, on the device of `starts`.

    starts / blocks / targets: [N, 7] float64.  noise: [N, AUG_NOISE_ROWS, 7] uniform draws in the
    reference's per-trajectory order (pick, down, grab, up, place, descend, drop), e.g.
    np.random.rand(N * 7500 * 7) for a seeded reference run, or torch.rand on the GPU.
    `traj` is the time-major [AUG_T, N, 7] table (2.4 GB at N = 4096: resident in HBM), and
    traj[:, i] equals the reference's trajectory for (starts[i], [blocks[i], targets[i]]) bit-for-bit.
    """

    def __init__(self, starts, blocks, targets, noise):
        import torch
        dev = starts.device
        f64 = dict(dtype=torch.float64, device=dev)
        n = starts.shape[0]
        tt = torch.from_numpy(np.linspace(0, 1, NUM_POINTS + 1)[1:]).to(dev)
        noise = noise.to(**f64)
        assert noise.shape == (n, AUG_NOISE_ROWS, 7)
        self.T = AUG_T
        self.traj = torch.empty((AUG_T, n, 7), **f64)
        off = 0

        def seg(k, a, b):
            nonlocal off
            norm, nrows = AUG_NOISE[k]
            slope = (b - a) / (1.0 - 0.0)
            pts = slope[None] * (tt[:, None, None] - 0.0) + a[None]      # [15, N, 7]
            pts[-1] = b                                                  # np.interp hits `stop` exactly
            rows = pts.repeat_interleave(AUG_HOLD, dim=0)                # [1500, N, 7]
            nz = torch.zeros_like(rows)
            nz[:nrows] = noise[:, off:off + nrows].transpose(0, 1) / norm
            off += nrows
            out = self.traj[k * AUG_SEG_ROWS:(k + 1) * AUG_SEG_ROWS]
            torch.add(rows, nz, out=out)
            return out[-1]

        def col(x, k, v):
            y = x.clone()
            y[:, k] = v
            return y

        e = seg(0, starts, col(blocks, 2, starts[:, 2]))
        e = seg(1, e, col(e, 2, blocks[:, 2]))
        e = seg(2, e, col(e, 6, 1.0))
        dz = torch.tensor([0, 0, 0.15, 0, 0, 0, 0], **f64)
        e = seg(3, e, e + dz)
        pl = targets.clone()
        pl[:, 2] = e[:, 2]
        e = seg(4, e, pl)
        dz = torch.tensor([0, 0, 0.025, 0, 0, 0, 0], **f64)
        e = seg(5, e, targets + dz)
        seg(6, e, col(e, 6, 0.0))

    def row(self, t: int):
        return self.traj[t]


class PickPlaceTorch:
    """Per-env build_traj_l_pick_place rows evaluated on the GPU: row(t) for all envs.

    starts/picks/places: [N, 7] float64 tensors.  Row t (0 <= t < 7200) equals
    build_traj_l_pick_place(start_i, [pick_i, place_i])[t] bit-for-bit.
    """

    def __init__(self, starts, picks, places):
        import torch
        self.torch = torch
        dev = starts.device
        dz = torch.tensor([0, 0, 0.025, 0, 0, 0, 0], dtype=torch.float64, device=dev)
        self.t = torch.from_numpy(np.linspace(0, 1, NUM_POINTS + 1)).to(dev)
        places = places + dz
        # np.interp returns the segment end exactly at t == 1
        end_pick = picks
        up = end_pick.clone()
        up[:, 2] = end_pick[:, 2] + 0.15
        up[:, 6] = end_pick[:, 6] + (1 - end_pick[:, 6])
        end_up = up
        end_place = places
        drop = end_place.clone()
        drop[:, 6] = 0.0
        self.A = torch.stack([starts, end_pick, end_up, end_place])  # [4, N, 7]
        self.B = torch.stack([picks, up, places, drop])
        self.T = 4 * NUM_POINTS * HOLD_PICK_PLACE

    def row(self, t: int):
        seg = t // (NUM_POINTS * HOLD_PICK_PLACE)
        k = (t % (NUM_POINTS * HOLD_PICK_PLACE)) // HOLD_PICK_PLACE
        a, b = self.A[seg], self.B[seg]
        if k + 1 == NUM_POINTS:
            return b.clone()
        slope = (b - a) / (1.0 - 0.0)
        return slope * (self.t[k + 1] - 0.0) + a
