/*
 * ur3e_cvx_wave.h — the convex-mesh narrowphase of convex.h run by a whole 64-lane wavefront, for the
 * overlaid (compact and grasp) tiers of main.xml with its meshes.
 *
 * convex.h runs plane–convex, GJK and EPA as scalar code, one candidate pair per lane: its support
 * function walks the hull's vertices one by one, and its simplex and EPA polytope are private arrays
 * (scratch) -- in the compact tier that code spilled ~960 B per lane and ran each vertex loop on one lane
 * of the wave.  Here one wave settles one mesh pair at a time:
 *   - the hull vertices are lane-parallel: lane k holds vertex k in registers (vertices >= 64 are read
 *     from the model image), the support point is a wave argmax over the lanes' dot products (ties: the
 *     lowest vertex index, i.e. "the first vertex reaching the maximum" of convex.h's loop);
 *   - plane–convex computes every vertex distance at once and runs convex.h's keep-the-deepest selection
 *     over the vertices within the margin only;
 *   - the GJK simplex and the EPA polytope live in LDS (WCvxWork, in the overlaid layouts' narrowphase
 *     area), the scalar GJK/EPA logic runs on every lane alike (uniform control flow, no lane-restricted
 *     region), and EPA's per-face work (closest face, faces visible from the new vertex, the horizon's new
 *     faces) is lane-parallel over the faces, with convex.h's orders kept where they decide a result: the
 *     horizon edge list is built face by face in convex.h's order, new faces take indices in edge order,
 *     and the closest face is the first minimal one.
 * Every number is computed by the same expression, operand for operand, as in convex.h (both sides build
 * with -ffp-contract=off), so a pair's contacts are bit-identical to the oracle's and to the full-capacity
 * tier's.  The wave's EPA holds convex.h's capacities (UR3E_EPA_MAXV vertices, UR3E_EPA_MAXF faces) but at
 * most WC_MAXE horizon edges per step; more hands the env-step on (ovf) to the full-capacity tier.
 */
#ifndef UR3E_CVX_WAVE_H
#define UR3E_CVX_WAVE_H

/* included from ur3e_wave.h after ur3e_wave_r.h (needs WD, w_lane, rl) */

/* WCvxWork, WMeshRes and the WC_ capacities are declared in ur3e_wave.h (the overlaid layouts hold them) */

/* a geom as a convex shape: uniform part (pose, box half sizes or hull) ... */
struct WCvxShape {
  double pos[3], mat[9], size[3];
  const double* v; /* hull vertices (model image) or null: a box */
  int nv;
};
/* ... and this lane's hull vertex (lane k: vertex k, k < 64) */
struct WCvxLane {
  double x, y, z;
};

template <class KS>
__device__ __forceinline__ void wc_shape(KModel m, const KS& s, int g, WCvxShape& c, WCvxLane& lv) {
  const int lane = w_lane();
  if (m->geom_type[g] == UR3E_GEOM_MESH) {
    const int id = m->geom_dataid[g];
    c.v = &m->mesh_vert[m->mesh_vertadr[id]][0];
    c.nv = m->mesh_vertnum[id];
  } else {
    c.v = nullptr;
    c.nv = 0;
  }
#pragma unroll
  for (int k = 0; k < 3; k++) { c.size[k] = m->geom_size[g][k]; c.pos[k] = s.geom_xpos[g][k]; }
#pragma unroll
  for (int k = 0; k < 9; k++) c.mat[k] = s.geom_xmat[g][k];
  lv.x = 0; lv.y = 0; lv.z = 0;
  if (lane < c.nv) {
    lv.x = c.v[3 * lane]; lv.y = c.v[3 * lane + 1]; lv.z = c.v[3 * lane + 2];
  }
}

WD double wc_shfx(double v, int mask) { return __shfl_xor(v, mask); }

/* wave argmax of (val, idx): the largest val, ties to the lowest idx (every lane gets the winner) */
WD int wc_argmax(double val, int idx) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const double ov = wc_shfx(val, off);
    const int oi = __shfl_xor(idx, off);
    const bool take = ov > val || (ov == val && oi < idx);
    val = take ? ov : val;
    idx = take ? oi : idx;
  }
  return idx;
}
/* wave argmin of (val, idx): the smallest val, ties to the lowest idx */
WD int wc_argmin(double val, int idx) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const double ov = wc_shfx(val, off);
    const int oi = __shfl_xor(idx, off);
    const bool take = ov < val || (ov == val && oi < idx);
    val = take ? ov : val;
    idx = take ? oi : idx;
  }
  return idx;
}

/* vertex k (wave-uniform) of a hull */
WD void wc_vertex(const WCvxShape& c, const WCvxLane& lv, int k, double out[3]) {
  if (k < 64) {
    out[0] = rl(lv.x, k); out[1] = rl(lv.y, k); out[2] = rl(lv.z, k);
  } else {
    out[0] = c.v[3 * k]; out[1] = c.v[3 * k + 1]; out[2] = c.v[3 * k + 2];
  }
}

/* ur3e_cvx_support: the support point of shape c in world direction d (wave-uniform d and result) */
WD void wc_support(const WCvxShape& c, const WCvxLane& lv, const double d[3], double out[3]) {
  const double* R = c.mat;
  const double ld0 = R[0] * d[0] + R[3] * d[1] + R[6] * d[2];
  const double ld1 = R[1] * d[0] + R[4] * d[1] + R[7] * d[2];
  const double ld2 = R[2] * d[0] + R[5] * d[1] + R[8] * d[2];
  double l0, l1, l2;
  if (c.v) {
    const int lane = w_lane();
    /* convex.h keeps the first vertex reaching the maximum and skips a NaN product (a NaN at vertex 0
       keeps vertex 0): a NaN counts as -inf in the argmax, and vertex 0's NaN decides alone */
    double dd = -__builtin_inf();
    int idx = 0x7fffffff;
    bool nan0 = false;
    for (int base = 0; base < c.nv; base += 64) {
      const int k = base + lane;
      if (k < c.nv) {
        double x, y, z;
        if (base == 0) { x = lv.x; y = lv.y; z = lv.z; }
        else { x = c.v[3 * k]; y = c.v[3 * k + 1]; z = c.v[3 * k + 2]; }
        double e = x * ld0 + y * ld1 + z * ld2;
        if (k == 0) nan0 = e != e;
        if (e != e) e = -__builtin_inf();
        if (e > dd || idx == 0x7fffffff) { dd = e; idx = k; } /* chunks ascend: ties keep the earlier */
      }
    }
    int best = wc_argmax(dd, idx);
    if (__ballot(nan0) != 0) best = 0;
    double vb[3];
    wc_vertex(c, lv, best, vb);
    l0 = vb[0]; l1 = vb[1]; l2 = vb[2];
  } else {
    l0 = ld0 >= 0 ? c.size[0] : -c.size[0];
    l1 = ld1 >= 0 ? c.size[1] : -c.size[1];
    l2 = ld2 >= 0 ? c.size[2] : -c.size[2];
  }
  out[0] = c.pos[0] + R[0] * l0 + R[1] * l1 + R[2] * l2;
  out[1] = c.pos[1] + R[3] * l0 + R[4] * l1 + R[5] * l2;
  out[2] = c.pos[2] + R[6] * l0 + R[7] * l1 + R[8] * l2;
}

/* ur3e_mink_support */
WD void wc_mink(const WCvxShape& A, const WCvxLane& la, const WCvxShape& B, const WCvxLane& lb, const double d[3],
                double a[3], double b[3], double w[3]) {
  const double nd[3] = {-d[0], -d[1], -d[2]};
  wc_support(A, la, d, a);
  wc_support(B, lb, nd, b);
  ur3e_cvx_sub(w, a, b);
}

/* ---- plane (geom1) vs convex hull (geom2) ---------------------------------------------------- */
/* signed distances of this lane's vertices (chunk `base`) from the plane: d0 + n . (R v), convex.h's
   expressions */
WD double wc_plane_dist(const double n[3], double d0, const WCvxShape& c, double x, double y, double z) {
  const double* R = c.mat;
  double w[3];
  w[0] = R[0] * x + R[1] * y + R[2] * z;
  w[1] = R[3] * x + R[4] * y + R[5] * z;
  w[2] = R[6] * x + R[7] * y + R[8] * z;
  return d0 + ur3e_cvx_dot(n, w);
}

/* ur3e_plane_convex: up to UR3E_CVX_PLANE_MAX contacts into res (count returned) */
WD int wc_plane_convex(const double pp[3], const double pm[9], const WCvxShape& c, const WCvxLane& lv,
                       double margin, WCvxWork& W, double (*res)[7], int room) {
  const double n[3] = {pm[2], pm[5], pm[8]};
  double dif[3];
  ur3e_cvx_sub(dif, c.pos, pp);
  const double d0 = ur3e_cvx_dot(n, dif);
  const int lane = w_lane();
  int ns = 0;
  /* vertices within the margin, in vertex order, through convex.h's keep-the-deepest selection (run
     alike on every lane over the ballot of the chunk's near vertices) */
  for (int base = 0; base < c.nv; base += 64) {
    const int k = base + lane;
    double dd = 0;
    bool near = false;
    if (k < c.nv) {
      double x = lv.x, y = lv.y, z = lv.z;
      if (base) { x = c.v[3 * k]; y = c.v[3 * k + 1]; z = c.v[3 * k + 2]; }
      dd = wc_plane_dist(n, d0, c, x, y, z);
      near = !(dd > margin);
    }
    unsigned long long bm = __ballot(near);
    while (bm) {
      const int q = __builtin_ctzll(bm);
      bm &= bm - 1;
      const double ddq = rl(dd, q);
      const int kq = base + q;
      if (ns < UR3E_CVX_PLANE_MAX) {
        W.psel[ns] = kq; W.psd[ns] = ddq; ns++;
      } else {
        int worst = 0;
        for (int j = 1; j < ns; j++)
          if (W.psd[j] > W.psd[worst]) worst = j;
        if (ddq < W.psd[worst]) { W.psel[worst] = kq; W.psd[worst] = ddq; }
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
    }
  }
  const double* R = c.mat;
  for (int i = 0; i < ns; i++) {
    int b = i;
    for (int j = i + 1; j < ns; j++)
      if (W.psd[j] < W.psd[b] || (W.psd[j] == W.psd[b] && W.psel[j] < W.psel[b])) b = j;
    const int tk = W.psel[i], bk = W.psel[b];
    const double td = W.psd[i], bd = W.psd[b];
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    W.psel[i] = bk; W.psel[b] = tk;
    W.psd[i] = bd; W.psd[b] = td;
    double v[3];
    wc_vertex(c, lv, bk, v);
    double w[3];
    w[0] = R[0] * v[0] + R[1] * v[1] + R[2] * v[2];
    w[1] = R[3] * v[0] + R[4] * v[1] + R[5] * v[2];
    w[2] = R[6] * v[0] + R[7] * v[1] + R[8] * v[2];
    const double h = bd * 0.5;
    if (i < room) {
      res[i][0] = c.pos[0] + w[0] - n[0] * h;
      res[i][1] = c.pos[1] + w[1] - n[1] * h;
      res[i][2] = c.pos[2] + w[2] - n[2] * h;
      res[i][3] = n[0]; res[i][4] = n[1]; res[i][5] = n[2];
      res[i][6] = bd;
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
  }
  return ns;
}

/* ---- GJK on the Minkowski difference A - B (simplex in LDS) --------------------------------- */
/* keep simplex entries (i0, i1, i2)[:n] in that order (convex.h ur3e_simplex_keep) */
WD void wc_keep(WCvxWork& W, int i0, int i1, int i2, int n) {
  double t[3][9];
  const int idx[3] = {i0, i1, i2};
#pragma unroll
  for (int k = 0; k < 3; k++)
#pragma unroll
    for (int c = 0; c < 3; c++) {
      t[k][c] = W.sw[idx[k]][c]; t[k][3 + c] = W.sa[idx[k]][c]; t[k][6 + c] = W.sb[idx[k]][c];
    }
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
#pragma unroll
  for (int k = 0; k < 3; k++)
    if (k < n) {
#pragma unroll
      for (int c = 0; c < 3; c++) { W.sw[k][c] = t[k][c]; W.sa[k][c] = t[k][3 + c]; W.sb[k][c] = t[k][6 + c]; }
    }
  W.sn = n;
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

/* ur3e_sx_triangle on simplex entries (i0, i1, i2), without touching the simplex: the closest point v,
   the weights lam of the kept feature, and the feature as (nk, kk[]) = positions in (i0, i1, i2) */
WD void wc_tri(const WCvxWork& W, int i0, int i1, int i2, double v[3], double lam[3], int& nk, int kk[3]) {
  double A[3], B[3], C[3];
#pragma unroll
  for (int c = 0; c < 3; c++) { A[c] = W.sw[i0][c]; B[c] = W.sw[i1][c]; C[c] = W.sw[i2][c]; }
  double ab[3], ac[3];
  ur3e_cvx_sub(ab, B, A); ur3e_cvx_sub(ac, C, A);
  const double ap[3] = {-A[0], -A[1], -A[2]};
  const double d1 = ur3e_cvx_dot(ab, ap), d2 = ur3e_cvx_dot(ac, ap);
  kk[0] = 0; kk[1] = 1; kk[2] = 2;
  lam[0] = 1; lam[1] = 0; lam[2] = 0;
  /* vertex q alone (ur3e_sx_vertex) */
#define WC_VTX(q, P)                                          \
  do {                                                        \
    nk = 1; kk[0] = q; lam[0] = 1;                            \
    v[0] = P[0]; v[1] = P[1]; v[2] = P[2];                    \
    return;                                                   \
  } while (0)
  /* edge (q, r) with parameter u (ur3e_sx_edge: w_q + u (w_r - w_q)) */
#define WC_EDGE(q, r, P, Q, u)                                \
  do {                                                        \
    const double uu = (u);                                    \
    nk = 2; kk[0] = q; kk[1] = r;                             \
    lam[0] = 1 - uu; lam[1] = uu;                             \
    for (int c = 0; c < 3; c++) v[c] = P[c] + uu * (Q[c] - P[c]); \
    return;                                                   \
  } while (0)
  if (d1 <= 0 && d2 <= 0) WC_VTX(0, A);
  const double bp[3] = {-B[0], -B[1], -B[2]};
  const double d3 = ur3e_cvx_dot(ab, bp), d4 = ur3e_cvx_dot(ac, bp);
  if (d3 >= 0 && d4 <= d3) WC_VTX(1, B);
  const double vc = d1 * d4 - d3 * d2;
  if (vc <= 0 && d1 >= 0 && d3 <= 0) WC_EDGE(0, 1, A, B, d1 / (d1 - d3));
  const double cp[3] = {-C[0], -C[1], -C[2]};
  const double d5 = ur3e_cvx_dot(ab, cp), d6 = ur3e_cvx_dot(ac, cp);
  if (d6 >= 0 && d5 <= d6) WC_VTX(2, C);
  const double vb = d5 * d2 - d1 * d6;
  if (vb <= 0 && d2 >= 0 && d6 <= 0) WC_EDGE(0, 2, A, C, d2 / (d2 - d6));
  const double va = d3 * d6 - d5 * d4;
  if (va <= 0 && (d4 - d3) >= 0 && (d5 - d6) >= 0) WC_EDGE(1, 2, B, C, (d4 - d3) / ((d4 - d3) + (d5 - d6)));
  const double den = va + vb + vc;
  if (!(den > 0)) {
    const double t = d1, dd = ur3e_cvx_dot(ab, ab);
    if (!(t > 0) || !(dd > 0)) WC_VTX(0, A);
    if (t >= dd) WC_VTX(1, B);
    WC_EDGE(0, 1, A, B, t / dd);
  }
  const double vv = vb / den, ww = vc / den;
  nk = 3;
  lam[0] = 1 - vv - ww; lam[1] = vv; lam[2] = ww;
  for (int c = 0; c < 3; c++) v[c] = A[c] + ab[c] * vv + ac[c] * ww;
#undef WC_VTX
#undef WC_EDGE
}

/* apply a wc_tri result on entries (i0, i1, i2) to the simplex */
WD void wc_apply_tri(WCvxWork& W, int i0, int i1, int i2, int nk, const int kk[3], const double lam[3]) {
  const int src[3] = {i0, i1, i2};
  int j[3];
#pragma unroll
  for (int q = 0; q < 3; q++) j[q] = kk[q] == 0 ? src[0] : (kk[q] == 1 ? src[1] : src[2]);
  wc_keep(W, j[0], j[1], j[2], nk);
  W.slam[0] = lam[0]; W.slam[1] = lam[1]; W.slam[2] = lam[2];
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

/* ur3e_simplex_closest: closest point v of the simplex, reduced to its supporting feature (weights in
   W.slam); 1 when the origin lies inside the tetrahedron */
WD int wc_closest(WCvxWork& W, double v[3]) {
  const int n = W.sn;
  if (n == 1) {
    v[0] = W.sw[0][0]; v[1] = W.sw[0][1]; v[2] = W.sw[0][2];
    W.slam[0] = 1;
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    return 0;
  }
  if (n == 2) {
    double w0[3], w1[3], ab[3];
#pragma unroll
    for (int c = 0; c < 3; c++) { w0[c] = W.sw[0][c]; w1[c] = W.sw[1][c]; }
    ur3e_cvx_sub(ab, w1, w0);
    const double ao[3] = {-w0[0], -w0[1], -w0[2]};
    const double t = ur3e_cvx_dot(ao, ab), dd = ur3e_cvx_dot(ab, ab);
    if (!(t > 0) || !(dd > 0)) {
      wc_keep(W, 0, 0, 0, 1);
      v[0] = w0[0]; v[1] = w0[1]; v[2] = w0[2];
      W.slam[0] = 1;
    } else if (t >= dd) {
      wc_keep(W, 1, 0, 0, 1);
      v[0] = w1[0]; v[1] = w1[1]; v[2] = w1[2];
      W.slam[0] = 1;
    } else {
      const double u = t / dd;
      W.slam[0] = 1 - u; W.slam[1] = u;
      for (int c = 0; c < 3; c++) v[c] = w0[c] + u * (w1[c] - w0[c]);
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    return 0;
  }
  if (n == 3) {
    double lam[3];
    int nk, kk[3];
    wc_tri(W, 0, 1, 2, v, lam, nk, kk);
    wc_apply_tri(W, 0, 1, 2, nk, kk, lam);
    return 0;
  }
  /* tetrahedron */
  const int F[4][4] = {{0, 1, 2, 3}, {0, 3, 1, 2}, {0, 2, 3, 1}, {1, 3, 2, 0}};
  double best = 1e300;
  int bf = -1, bnk = 0, bkk[3] = {0, 1, 2};
  double bv[3] = {0, 0, 0}, bl[3] = {0, 0, 0};
#pragma unroll
  for (int f = 0; f < 4; f++) {
    double A[3], B[3], C[3], D[3];
#pragma unroll
    for (int c = 0; c < 3; c++) {
      A[c] = W.sw[F[f][0]][c]; B[c] = W.sw[F[f][1]][c]; C[c] = W.sw[F[f][2]][c]; D[c] = W.sw[F[f][3]][c];
    }
    double ab[3], ac[3], nn[3], ad[3];
    ur3e_cvx_sub(ab, B, A); ur3e_cvx_sub(ac, C, A); ur3e_cvx_cross(nn, ab, ac);
    ur3e_cvx_sub(ad, D, A);
    const double sd = ur3e_cvx_dot(nn, ad);
    const double so = -ur3e_cvx_dot(nn, A);
    if (sd * so < 0 || sd == 0) {
      double tv[3], tl[3];
      int nk, kk[3];
      wc_tri(W, F[f][0], F[f][1], F[f][2], tv, tl, nk, kk);
      const double dd = ur3e_cvx_dot(tv, tv);
      if (dd < best) {
        best = dd; bf = f; bnk = nk;
        bkk[0] = kk[0]; bkk[1] = kk[1]; bkk[2] = kk[2];
        bv[0] = tv[0]; bv[1] = tv[1]; bv[2] = tv[2];
        bl[0] = tl[0]; bl[1] = tl[1]; bl[2] = tl[2];
      }
    }
  }
  if (bf < 0) {
    v[0] = 0; v[1] = 0; v[2] = 0;
    return 1;
  }
  int f0 = 0, f1 = 1, f2 = 2;
#pragma unroll
  for (int f = 1; f < 4; f++)
    if (bf == f) { f0 = F[f][0]; f1 = F[f][1]; f2 = F[f][2]; }
  wc_apply_tri(W, f0, f1, f2, bnk, bkk, bl);
  v[0] = bv[0]; v[1] = bv[1]; v[2] = bv[2];
  return 0;
}

/* ur3e_gjk (convex.h, the same early exit: 2 when a support point proves the hulls farther apart than cut) */
WD int wc_gjk(const WCvxShape& A, const WCvxLane& la, const WCvxShape& B, const WCvxLane& lb, WCvxWork& W,
              double pa[3], double pb[3], double cut = -1.0) {
  double d[3];
  ur3e_cvx_sub(d, B.pos, A.pos);
  d[0] = -d[0]; d[1] = -d[1]; d[2] = -d[2];
  if (d[0] == 0 && d[1] == 0 && d[2] == 0) d[0] = 1;
  double a[3], b[3], w[3];
  wc_mink(A, la, B, lb, d, a, b, w);
#pragma unroll
  for (int c = 0; c < 3; c++) { W.sw[0][c] = w[c]; W.sa[0][c] = a[c]; W.sb[0][c] = b[c]; }
  W.sn = 1;
  W.slam[0] = 1; W.slam[1] = 0; W.slam[2] = 0; W.slam[3] = 0;
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  double v[3] = {w[0], w[1], w[2]};
  for (int it = 0; it < UR3E_GJK_ITERS; it++) {
    const double vv = ur3e_cvx_dot(v, v);
    if (vv <= 1e-30) return 1;
    const double nd[3] = {-v[0], -v[1], -v[2]};
    wc_mink(A, la, B, lb, nd, a, b, w);
    const double vw = ur3e_cvx_dot(v, w);
    if (cut >= 0 && vw > 0 && vw * vw > cut * cut * vv) return 2; /* apart beyond cut */
    if (vv - vw <= UR3E_GJK_TOL * vv) break;
    const int k = W.sn;
#pragma unroll
    for (int c = 0; c < 3; c++) { W.sw[k][c] = w[c]; W.sa[k][c] = a[c]; W.sb[k][c] = b[c]; }
    W.sn = k + 1;
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    if (wc_closest(W, v)) return 1;
  }
  const int n = W.sn;
  for (int c = 0; c < 3; c++) {
    double xa = 0, xb = 0;
    for (int k = 0; k < n; k++) { xa += W.slam[k] * W.sa[k][c]; xb += W.slam[k] * W.sb[k][c]; }
    pa[c] = xa; pb[c] = xb;
  }
  return 0;
}

/* ---- EPA (polytope in LDS, per-face work lane-parallel) ------------------------------------- */
WD void wc_pw(const WCvxWork& W, int i, double w[3]) {
  double a[3], b[3];
#pragma unroll
  for (int c = 0; c < 3; c++) { a[c] = W.pa[i][c]; b[c] = W.pb[i][c]; }
  ur3e_cvx_sub(w, a, b);
}

/* ur3e_epa_face's arithmetic for face (i, j, k): unit normal n and offset d; false when degenerate.
   orient = 1 winds it away from the origin (swap reports the (i, k, j) winding) */
WD bool wc_face_calc(const WCvxWork& W, int i, int j, int k, int orient, double n[3], double& d, bool& swap) {
  double wi[3], wj[3], wk[3], ab[3], ac[3];
  wc_pw(W, i, wi); wc_pw(W, j, wj); wc_pw(W, k, wk);
  ur3e_cvx_sub(ab, wj, wi);
  ur3e_cvx_sub(ac, wk, wi);
  ur3e_cvx_cross(n, ab, ac);
  const double len = sqrt(ur3e_cvx_dot(n, n));
  swap = false;
  if (!(len > 0)) return false;
  n[0] /= len; n[1] /= len; n[2] /= len;
  d = ur3e_cvx_dot(n, wi);
  if (orient && d < 0) {
    n[0] = -n[0]; n[1] = -n[1]; n[2] = -n[2];
    d = -d;
    swap = true;
  }
  return true;
}

/* one face added by every lane alike (the initial tetrahedron) */
WD bool wc_face1(WCvxWork& W, int i, int j, int k) {
  const int f = W.pnf;
  if (f >= WC_MAXF) return false;
  double n[3], d;
  bool swap;
  if (!wc_face_calc(W, i, j, k, 1, n, d, swap)) return false;
  W.fv[f] = swap ? (i | k << 8 | j << 16 | 1 << 24) : (i | j << 8 | k << 16 | 1 << 24);
  W.fn[f][0] = n[0]; W.fn[f][1] = n[1]; W.fn[f][2] = n[2];
  W.fd[f] = d;
  W.pnf = f + 1;
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  return true;
}

/* grow a GJK simplex of 1-3 points to a tetrahedron (ur3e_epa_seed) */
WD bool wc_epa_seed(const WCvxShape& A, const WCvxLane& la, const WCvxShape& B, const WCvxLane& lb, WCvxWork& W) {
  for (int q = 0; q < 6 && W.sn < 4; q++) {
    /* convex.h's directions {+x, -x, +y, -y, +z, -z} (exact constants, +0 elsewhere) */
    const double sg = (q & 1) ? -1.0 : 1.0;
    const double dq[3] = {(q >> 1) == 0 ? sg : 0.0, (q >> 1) == 1 ? sg : 0.0, (q >> 1) == 2 ? sg : 0.0};
    double a[3], b[3], w[3];
    wc_mink(A, la, B, lb, dq, a, b, w);
    const int n = W.sn;
    int dup = 0;
    for (int k = 0; k < n; k++) {
      double e[3], sk[3] = {W.sw[k][0], W.sw[k][1], W.sw[k][2]};
      ur3e_cvx_sub(e, w, sk);
      if (ur3e_cvx_dot(e, e) < 1e-24) dup = 1;
    }
    double s0[3] = {W.sw[0][0], W.sw[0][1], W.sw[0][2]}, s1[3] = {W.sw[1][0], W.sw[1][1], W.sw[1][2]};
    if (n == 2 && !dup) {
      double e1[3], e2[3], cr[3];
      ur3e_cvx_sub(e1, s1, s0); ur3e_cvx_sub(e2, w, s0); ur3e_cvx_cross(cr, e1, e2);
      if (ur3e_cvx_dot(cr, cr) < 1e-24) dup = 1;
    }
    if (n == 3 && !dup) {
      double s2[3] = {W.sw[2][0], W.sw[2][1], W.sw[2][2]};
      double e1[3], e2[3], e3[3], cr[3];
      ur3e_cvx_sub(e1, s1, s0); ur3e_cvx_sub(e2, s2, s0); ur3e_cvx_sub(e3, w, s0);
      ur3e_cvx_cross(cr, e1, e2);
      const double vol = ur3e_cvx_dot(cr, e3);
      if (vol * vol < 1e-36) dup = 1;
    }
    if (dup) continue;
#pragma unroll
    for (int c = 0; c < 3; c++) { W.sw[n][c] = w[c]; W.sa[n][c] = a[c]; W.sb[n][c] = b[c]; }
    W.sn = n + 1;
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
  }
  return W.sn == 4;
}

/* the closest alive face (convex.h: the first alive face with the smallest fd, NaN never smaller; a NaN
   on the first alive face keeps it), or -1 */
WD int wc_best_face(const WCvxWork& W) {
  const int lane = w_lane();
  const int nf = W.pnf;
  double key = __builtin_inf();
  int idx = 0x7fffffff;
  int first = 0x7fffffff;
  bool any = false;
#pragma unroll
  for (int sl = 0; sl < WC_FSLOT; sl++) {
    const int f = sl * 64 + lane;
    if (f < nf && (W.fv[f] >> 24 & 1)) {
      double x = W.fd[f];
      any = true;
      if (f < first) first = f;
      if (x != x) x = __builtin_inf();
      if (x < key || idx == 0x7fffffff) { key = x; idx = f; }
    }
  }
  if (__ballot(any) == 0) return -1;
  const int best = wc_argmin(key, idx);
  int fa = first;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const int o = __shfl_xor(fa, off);
    fa = o < fa ? o : fa;
  }
  const double d0 = W.fd[fa];
  return d0 != d0 ? fa : best;
}

/* ur3e_epa_run: 1 with the normal n (A to B), depth and witness points; 0 when EPA gives up; -1 when
   the horizon outgrew WC_MAXE (the env-step is handed on) */
WD int wc_epa(const WCvxShape& A, const WCvxLane& la, const WCvxShape& B, const WCvxLane& lb, WCvxWork& W,
              double n[3], double* depth, double pa[3], double pb[3]) {
  const int lane = w_lane();
  if (W.sn < 4 && !wc_epa_seed(A, la, B, lb, W)) return 0;
  /* the simplex's four points become the polytope's first vertices (w = a - b as stored) */
  if (lane < 12) {
    const int k = lane / 3, c = lane % 3;
    W.pa[k][c] = W.sa[k][c];
    W.pb[k][c] = W.sb[k][c];
  }
  W.pnv = 4;
  W.pnf = 0;
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  if (!wc_face1(W, 0, 1, 2) || !wc_face1(W, 0, 3, 1) || !wc_face1(W, 0, 2, 3) || !wc_face1(W, 1, 3, 2)) return 0;
  int best = 0;
  for (int it = 0; it < UR3E_EPA_ITERS; it++) {
    best = wc_best_face(W);
    if (best < 0) return 0;
    const double fnb[3] = {W.fn[best][0], W.fn[best][1], W.fn[best][2]};
    double a[3], b[3], w[3];
    wc_mink(A, la, B, lb, fnb, a, b, w);
    const double dw = ur3e_cvx_dot(fnb, w);
    if (dw - W.fd[best] <= UR3E_EPA_TOL) break;
    if (W.pnv >= WC_MAXV) break;
    const int nvx = W.pnv;
    if (lane < 3) {
      W.pa[nvx][lane] = lane == 0 ? a[0] : (lane == 1 ? a[1] : a[2]);
      W.pb[nvx][lane] = lane == 0 ? b[0] : (lane == 1 ? b[1] : b[2]);
    }
    W.pnv = nvx + 1;
    /* faces that see w (lane-parallel over the faces present when the step began) */
    const int nf = W.pnf;
    unsigned long long rm[WC_FSLOT];
#pragma unroll
    for (int sl = 0; sl < WC_FSLOT; sl++) {
      const int f = sl * 64 + lane;
      bool see = false;
      if (f < nf) {
        const int fv = W.fv[f];
        if (fv >> 24 & 1) {
          double w0[3], dv[3];
          wc_pw(W, fv & 0xff, w0);
          ur3e_cvx_sub(dv, w, w0);
          const double fnf[3] = {W.fn[f][0], W.fn[f][1], W.fn[f][2]};
          see = !(ur3e_cvx_dot(fnf, dv) <= 0);
        }
      }
      rm[sl] = __ballot(see);
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    /* the horizon: edges of exactly one removed face, in convex.h's list order (removed faces in index
       order, their edges in winding order; an edge whose reverse is listed cancels it, the list's last
       entry moving into its place) */
    int ne = 0;
    bool over = false;
#pragma unroll
    for (int sl = 0; sl < WC_FSLOT; sl++) {
      unsigned long long bm = rm[sl];
      while (bm) {
        const int f = sl * 64 + __builtin_ctzll(bm);
        bm &= bm - 1;
        const int fv = W.fv[f];
        if (lane == 0) W.fv[f] = fv & 0xffffff;
        const int vi[3] = {fv & 0xff, fv >> 8 & 0xff, fv >> 16 & 0xff};
#pragma unroll
        for (int e = 0; e < 3; e++) {
          const int i = vi[e], j = vi[(e + 1) % 3];
          const int rev = j | i << 8;
          const unsigned long long hit = __ballot(lane < ne && W.edge[lane < WC_MAXE ? lane : 0] == rev);
          if (hit) {
            const int q = 63 - __builtin_clzll(hit);
            const int last = W.edge[ne - 1];
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
            if (lane == 0) W.edge[q] = last;
            ne--;
          } else if (ne < WC_MAXE) {
            if (lane == 0) W.edge[ne] = i | j << 8;
            ne++;
          } else {
            over = true;
          }
          __builtin_amdgcn_wave_barrier();
          asm volatile("" ::: "memory");
        }
      }
    }
    /* convex.h's list holds 3 * UR3E_EPA_MAXF edges: outgrowing ours means its result is not ours */
    if (over) return -1;
    /* new faces (edge i, edge j, new vertex), lane q for horizon edge q; indices in edge order, none
       past the capacity (convex.h's ur3e_epa_face refuses a degenerate face and a full list) */
    bool okf = false;
    double fnq[3] = {0, 0, 0}, fdq = 0;
    int fvq = 0;
    if (lane < ne) {
      const int eq = W.edge[lane];
      bool swap;
      okf = wc_face_calc(W, eq & 0xff, eq >> 8 & 0xff, nvx, 0, fnq, fdq, swap);
      fvq = (eq & 0xff) | (eq >> 8 & 0xff) << 8 | nvx << 16 | 1 << 24;
    }
    const unsigned long long okb = __ballot(okf);
    const int before = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(okb >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)okb, 0u));
    const int fi = nf + before;
    const bool put = okf && fi < WC_MAXF;
    if (put) {
      W.fv[fi] = fvq;
      W.fn[fi][0] = fnq[0]; W.fn[fi][1] = fnq[1]; W.fn[fi][2] = fnq[2];
      W.fd[fi] = fdq;
    }
    const int added = __popcll(__ballot(put));
    W.pnf = nf + added;
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    if (added != ne) break; /* some face refused: convex.h stops after adding the others */
  }
  best = wc_best_face(W);
  if (best < 0) return 0;
  const int fv = W.fv[best];
  const int i0 = fv & 0xff, i1 = fv >> 8 & 0xff, i2 = fv >> 16 & 0xff;
  const double fnb[3] = {W.fn[best][0], W.fn[best][1], W.fn[best][2]};
  const double fdb = W.fd[best];
  double p[3] = {fnb[0] * fdb, fnb[1] * fdb, fnb[2] * fdb};
  double w0[3], w1[3], w2[3], v0[3], v1[3], v2[3];
  wc_pw(W, i0, w0); wc_pw(W, i1, w1); wc_pw(W, i2, w2);
  ur3e_cvx_sub(v0, w1, w0); ur3e_cvx_sub(v1, w2, w0); ur3e_cvx_sub(v2, p, w0);
  const double d00 = ur3e_cvx_dot(v0, v0), d01 = ur3e_cvx_dot(v0, v1), d11 = ur3e_cvx_dot(v1, v1);
  const double d20 = ur3e_cvx_dot(v2, v0), d21 = ur3e_cvx_dot(v2, v1);
  const double den = d00 * d11 - d01 * d01;
  double l1 = 0, l2 = 0;
  if (den > 0) { l1 = (d11 * d20 - d01 * d21) / den; l2 = (d00 * d21 - d01 * d20) / den; }
  const double l0 = 1 - l1 - l2;
  for (int c = 0; c < 3; c++) {
    pa[c] = l0 * W.pa[i0][c] + l1 * W.pa[i1][c] + l2 * W.pa[i2][c];
    pb[c] = l0 * W.pb[i0][c] + l1 * W.pb[i1][c] + l2 * W.pb[i2][c];
  }
  n[0] = fnb[0]; n[1] = fnb[1]; n[2] = fnb[2];
  *depth = fdb;
  return 1;
}

/* ur3e_convex_convex: 0 or 1 contact into res[0]; -1: hand the env-step on */
WD int wc_convex_convex(const WCvxShape& A, const WCvxLane& la, const WCvxShape& B, const WCvxLane& lb,
                        WCvxWork& W, double margin, double* res) {
  double pa[3], pb[3];
  const int g = wc_gjk(A, la, B, lb, W, pa, pb, margin + UR3E_GJK_CUT_SLACK);
  if (g == 2) return 0; /* apart beyond the margin: convex.h's no-contact answer */
  if (!g) {
    double dv[3];
    ur3e_cvx_sub(dv, pb, pa);
    const double dd = sqrt(ur3e_cvx_dot(dv, dv));
    if (!(dd <= margin) || !(dd > 0)) return 0;
    res[3] = dv[0] / dd; res[4] = dv[1] / dd; res[5] = dv[2] / dd;
    for (int c = 0; c < 3; c++) res[c] = 0.5 * (pa[c] + pb[c]);
    res[6] = dd;
    return 1;
  }
  double n[3], depth;
  const int r = wc_epa(A, la, B, lb, W, n, &depth, pa, pb);
  if (r <= 0) return r;
  res[3] = n[0]; res[4] = n[1]; res[5] = n[2];
  for (int c = 0; c < 3; c++) res[c] = 0.5 * (pa[c] + pb[c]);
  res[6] = -depth;
  return 1;
}

#endif /* UR3E_CVX_WAVE_H */
