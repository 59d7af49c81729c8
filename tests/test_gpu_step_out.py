"""GPU: Batch.step(out=...) writes the env-step's outputs into caller buffers -- here the views of one flat
payload, as bench.py's RCCL gather sends it (obs [n, 24] | reward [n] | terminated, truncated bytes) -- with
the same bits as the handle's own buffers, and refuses a wrong buffer before any launch."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_step_into_payload_views_bit_exact():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ur3e_amd import runtime as rt
    md, mc = rt.load_model("main_mesh")
    n, steps = 256, 40
    cfg = rt.make_config(task=rt.TASK_GYM_V2, frame_skip=2, model=md, seed=7, max_episode_steps=25)
    a_ref, b_out = rt.Batch(mc, cfg, n), rt.Batch(mc, cfg, n)
    od = b_out.obs_dim
    p = torch.full((n * od + n + (2 * n + 7) // 8,), float("nan"), dtype=torch.float64, device=b_out.device)
    fl = p[n * od + n:].view(torch.uint8)
    out = (p[:n * od].view(n, od), p[n * od:n * od + n], fl[:n], fl[n:2 * n])
    rng = np.random.default_rng(1)
    lo = np.array([0.04799994, -0.11650084, 0.0, 0.0])
    hi = np.array([0.54799994, 0.38349916, 0.5, 1.0])
    dones = 0
    for _ in range(steps):
        a = torch.from_numpy(rng.uniform(lo, hi, size=(n, 4)))
        r = a_ref.step(a)
        o = b_out.step(a, out=out)
        torch.cuda.synchronize()
        for x, y in zip(r[:4], o[:4]):
            assert torch.equal(x, y)
        assert torch.equal(r[4], o[4])  # terminal obs: the handle's own buffer either way
        dones += int((r[2] | r[3]).sum())
    assert dones > 0  # truncation at T = 25 crossed: the flags and terminal obs were exercised
    with pytest.raises(ValueError):
        b_out.step(a, out=(out[0], out[1].float(), out[2], out[3]))
    with pytest.raises(ValueError):
        b_out.step(a, out=(p[:n * od].view(od, n), out[1], out[2], out[3]))
    a_ref.close()
    b_out.close()
