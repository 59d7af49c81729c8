"""CPU: the C ABI's multi-rank gather (ur3e_gather_rows / ur3e_batch_gather, ur3e_amd/csrc/ur3e_gather.cpp)
with several ranks and no GPU.  The library's own code runs unchanged; only librccl is replaced, through
UR3E_RCCL_LIB, by tests/c/fake_rccl.c, whose point-to-point messages between processes go through files
(each receive checks its size against the matching send).  World sizes 2 and 4, every root: the root's
[nranks * n] buffers hold rank p's rows at [p * n, (p + 1) * n), obs, reward and both done flags; argument
errors come back as error codes before anything is sent.  The RCCL transport itself (xGMI, device
buffers, streams) is covered only at world size 1 on the GPU (tests/test_gpu_gather_rccl.py)."""
import ctypes
import multiprocessing as mp
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N, OD = 37, 24


def _fake_lib(tmp):
    so = os.path.join(tmp, "libfake_rccl.so")
    subprocess.run(["gcc", "-O1", "-shared", "-fPIC", "-o", so, os.path.join(REPO, "tests", "c", "fake_rccl.c")],
                   check=True)
    return so


def _payload(rank):
    rng = np.random.default_rng(100 + rank)
    obs = rng.standard_normal((N, OD)) + 1000.0 * rank
    rew = rng.standard_normal(N) - 10.0 * rank
    term = (rng.random(N) < 0.3).astype(np.uint8)
    trunc = ((rng.random(N) < 0.3) | (np.arange(N) == rank)).astype(np.uint8)
    return obs, rew, term, trunc


def _rank(rank, world, root, msgdir, fake, lib, q):
    try:
        os.environ["UR3E_RCCL_LIB"] = fake
        F = ctypes.CDLL(fake)
        F.fake_comm_init.restype = ctypes.c_void_p
        F.fake_comm_init.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_char_p]
        comm = ctypes.c_void_p(F.fake_comm_init(rank, world, msgdir.encode()))
        L = ctypes.CDLL(lib)
        L.ur3e_last_error.restype = ctypes.c_char_p
        vp = ctypes.c_void_p
        L.ur3e_gather_rows.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int] + [vp] * 9
        obs, rew, term, trunc = _payload(rank)
        p = lambda a: a.ctypes.data_as(vp)  # noqa: E731
        if rank == root:
            obs_all = np.full((world * N, OD), np.nan)
            rew_all = np.full(world * N, np.nan)
            term_all = np.full(world * N, 7, np.uint8)
            trunc_all = np.full(world * N, 7, np.uint8)
            bufs = [p(obs_all), p(rew_all), p(term_all), p(trunc_all)]
        else:
            bufs = [None] * 4
        # argument errors: nothing is sent (the later matched transfers would see stray messages otherwise)
        errs = [L.ur3e_gather_rows(comm, world, N, OD, p(obs), p(rew), p(term), p(trunc), *bufs, None),
                L.ur3e_gather_rows(comm, root, 0, OD, p(obs), p(rew), p(term), p(trunc), *bufs, None),
                L.ur3e_gather_rows(None, root, N, OD, p(obs), p(rew), p(term), p(trunc), *bufs, None)]
        if rank == root:
            errs.append(L.ur3e_gather_rows(comm, root, N, OD, p(obs), p(rew), p(term), p(trunc), None, None, None,
                                           None, None))
        rc = L.ur3e_gather_rows(comm, root, N, OD, p(obs), p(rew), p(term), p(trunc), *bufs, None)
        out = {"rank": rank, "rc": rc, "err": (L.ur3e_last_error() or b"").decode(), "errs": errs}
        if rank == root and rc == 0:
            out.update(obs=obs_all, rew=rew_all, term=term_all, trunc=trunc_all)
        q.put(out)
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put({"rank": rank, "rc": -99, "err": repr(e), "errs": []})


@pytest.mark.parametrize("world,root", [(2, 0), (2, 1), (4, 0), (4, 3)])
def test_gather_rows_rank_order(tmp_path, world, root):
    from ur3e_amd import runtime as rt
    lib = rt.LIB_PATH
    if not os.path.exists(lib):
        pytest.skip("library not built")
    fake = _fake_lib(str(tmp_path))
    msgdir = str(tmp_path / "msgs")
    os.makedirs(msgdir)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, world, root, msgdir, fake, lib, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = {}
    for _ in range(world):
        o = q.get(timeout=120)
        res[o["rank"]] = o
    for pr in procs:
        pr.join(60)
    for r in range(world):
        assert res[r]["rc"] == 0, res[r]["err"]
        assert all(e != 0 for e in res[r]["errs"]), res[r]["errs"]
    got = res[root]
    for r in range(world):
        obs, rew, term, trunc = _payload(r)
        sl = slice(r * N, (r + 1) * N)
        np.testing.assert_array_equal(got["obs"][sl], obs, err_msg=f"obs rows of rank {r}")
        np.testing.assert_array_equal(got["rew"][sl], rew, err_msg=f"reward rows of rank {r}")
        np.testing.assert_array_equal(got["term"][sl], term, err_msg=f"terminated rows of rank {r}")
        np.testing.assert_array_equal(got["trunc"][sl], trunc, err_msg=f"truncated rows of rank {r}")
    # each rank sent exactly its four messages (none on the error paths), each received once by the root
    left = [f for f in os.listdir(msgdir) if not f.endswith(".tmp")]
    assert len(left) == 4 * world
