"""GPU: ur3e_batch_gather (include/ur3e_batch.h, ur3e_amd/csrc/ur3e_gather.cpp), the C ABI's RCCL gather of
(obs, reward, terminated, truncated) to the policy rank, with a communicator the caller owns -- here a
world-size-1 RCCL communicator made through librccl's own C API (ncclGetUniqueId, ncclCommInitRank), as a
non-Python host would.  One GPU only: the gather to itself must deliver the step's buffers unchanged, in
the root's [nranks * n] layout; argument errors come back as error codes.  (Several ranks need several
GPUs; the torch.distributed path is covered over gloo in tests/test_sharded_gloo.py.)"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


class _UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]


def test_gather_to_self_through_a_caller_communicator():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ur3e_amd import runtime as rt
    torch.cuda.set_device(0)
    R = ctypes.CDLL("librccl.so.1")
    uid = _UniqueId()
    assert R.ncclGetUniqueId(ctypes.byref(uid)) == 0
    comm = ctypes.c_void_p()
    R.ncclCommInitRank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, _UniqueId, ctypes.c_int]
    assert R.ncclCommInitRank(ctypes.byref(comm), 1, uid, 0) == 0
    md, mc = rt.load_model("main")
    n = 512
    b = rt.Batch(mc, rt.make_config(task=rt.TASK_GYM_V2, frame_skip=2, model=md, seed=6, max_episode_steps=5), n)
    L = b.L
    vp = ctypes.c_void_p
    L.ur3e_batch_gather.argtypes = [vp, vp, ctypes.c_int] + [vp] * 9
    dev = b.device
    rng = np.random.default_rng(1)
    lo = np.array([0.04799994, -0.11650084, 0.0, 0.0])
    hi = np.array([0.54799994, 0.38349916, 0.5, 1.0])
    obs_all = torch.full((1 * n, b.obs_dim), -1.0, dtype=torch.float64, device=dev)
    rew_all = torch.full((1 * n,), -1.0, dtype=torch.float64, device=dev)
    term_all = torch.full((1 * n,), 7, dtype=torch.uint8, device=dev)
    trunc_all = torch.full((1 * n,), 7, dtype=torch.uint8, device=dev)
    stream = vp(torch.cuda.current_stream(dev).cuda_stream)
    truncs = 0
    for t in range(8):
        b.step(torch.from_numpy(rng.uniform(lo, hi, size=(n, 4))))
        rc = L.ur3e_batch_gather(b.h, comm, 0, vp(b.obs.data_ptr()), vp(b.reward.data_ptr()),
                                 vp(b.terminated.data_ptr()), vp(b.truncated.data_ptr()), vp(obs_all.data_ptr()),
                                 vp(rew_all.data_ptr()), vp(term_all.data_ptr()), vp(trunc_all.data_ptr()), stream)
        assert rc == 0, L.ur3e_last_error()
        torch.cuda.synchronize()
        assert torch.equal(obs_all, b.obs) and torch.equal(rew_all, b.reward)
        assert torch.equal(term_all, b.terminated) and torch.equal(trunc_all, b.truncated)
        truncs += int(b.truncated.sum().item())
    assert truncs > 0  # the done flags went through in both states
    # the root without its receive buffers, a root outside the communicator: errors, nothing enqueued
    null = vp()
    assert L.ur3e_batch_gather(b.h, comm, 0, vp(b.obs.data_ptr()), vp(b.reward.data_ptr()),
                               vp(b.terminated.data_ptr()), vp(b.truncated.data_ptr()), null, null, null, null,
                               stream) != 0
    assert L.ur3e_batch_gather(b.h, comm, 3, vp(b.obs.data_ptr()), vp(b.reward.data_ptr()),
                               vp(b.terminated.data_ptr()), vp(b.truncated.data_ptr()), vp(obs_all.data_ptr()),
                               vp(rew_all.data_ptr()), vp(term_all.data_ptr()), vp(trunc_all.data_ptr()),
                               stream) != 0
    b.close()
    R.ncclCommDestroy(comm)
