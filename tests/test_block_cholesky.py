"""The compact tier's block-diagonal Newton path (ur3e_wave_r.h r_direction, s.bdiag) skips the
cross block of H = M + J'DJ and the Cholesky updates that touch it.  The claim is exactness, signed
zeros included: with a +0 cross block (what the oracle's H build leaves there when no row couples
the two dof trees), the oracle's dense left-looking Cholesky (oracle/ur3e_oracle.c hessian_factor)
produces bit-for-bit the L of the skipping factorisation.  Checked here on the bit patterns (int64
views, so -0.0 != +0.0) of a numpy restatement of both loops, on random SPD blocks sized like main.xml
(arm + gripper 14 dofs, mug 6)."""
import numpy as np

MINVAL = 1e-15


def dense_chol(H):
    """oracle hessian_factor's Cholesky: column j, sum -= H[j][k]^2 (k < j), v -= H[i][k] H[j][k]"""
    H = H.copy()
    nv = H.shape[0]
    for j in range(nv):
        s = H[j, j]
        for k in range(j):
            s -= H[j, k] * H[j, k]
        if s < MINVAL:
            s = MINVAL
        ljj = np.sqrt(s)
        H[j, j] = ljj
        for i in range(j + 1, nv):
            v = H[i, j]
            for k in range(j):
                v -= H[i, k] * H[j, k]
            H[i, j] = v / ljj
    return np.tril(H)


def block_chol(H, split):
    """the kernel's block-diagonal variant: the cross block is the literal +0 and never updated"""
    nv = H.shape[0]
    L = np.zeros_like(H)
    for lo, hi in ((0, split), (split, nv)):
        L[lo:hi, lo:hi] = dense_chol(H[lo:hi, lo:hi])
    return L


def _spd_block(rng, n):
    A = rng.normal(size=(n, n))
    S = A @ A.T + n * np.eye(n)
    # exact zeros inside a block too (dofs that do not share a row), as in the tree-sparse mass matrix
    mask = rng.uniform(size=(n, n)) < 0.3
    mask = mask | mask.T
    np.fill_diagonal(mask, False)
    S[mask] = 0.0
    S += n * np.eye(n)
    return S


def test_block_cholesky_bit_identical():
    rng = np.random.default_rng(0)
    split, nv = 14, 20
    for _ in range(200):
        H = np.zeros((nv, nv))
        H[:split, :split] = _spd_block(rng, split)
        H[split:, split:] = _spd_block(rng, nv - split)
        # negative zeros where the oracle's J'DJ terms can leave them inside the blocks
        neg = rng.uniform(size=(nv, nv)) < 0.05
        H[neg & (H == 0)] = -0.0
        H[:split, split:] = 0.0
        H[split:, :split] = 0.0
        Ld = dense_chol(H)
        Lb = block_chol(H, split)
        assert np.array_equal(Ld.view(np.int64), Lb.view(np.int64))
