/*
 * ur3e_wave_r.h — register-resident Newton solver for the compact tier
 * (one 64-lane wavefront per env, nefc <= 64, nv <= K_NV <= 64).
 *
 * Same algorithm and the same floating-point operation order as w_solve_newton
 * (ur3e_wave.h) and the oracle's newton solver (oracle/ur3e_oracle.c), laid out
 * for the wavefront instead of LDS round trips:
 *   - lane r holds constraint row r: its Jacobian row, jar, force, state, cost
 *     terms; cone rows get their first row's zone/forces by a lane shuffle;
 *   - lane k holds dof k: qacc, Ma, grad, search, and row k of the Hessian
 *     (H build, right-looking Cholesky and the forward sweep stay in registers);
 *   - ordered reductions (costs, line-search sums, norms, gradient sums) walk
 *     the lanes in the oracle's order with v_readlane broadcasts;
 *   - LDS is read only for qM rows, J columns, the cone Hessians and L^T.
 * MuJoCo 3.3.3 semantics: engine_solver.c (mj_solNewton, Hessian/cone terms,
 * linesearch), engine_core_constraint.c (mj_constraintUpdate) as restated in
 * the oracle.
 */
#ifndef UR3E_WAVE_R_H
#define UR3E_WAVE_R_H

/* included from ur3e_wave.h (needs KSX, WD, WT) */

/* broadcast lane `lane` (wave-uniform) of v to every lane */
__device__ __forceinline__ double rl(double v, int lane) {
  long long b = __builtin_bit_cast(long long, v);
  int lo = __builtin_amdgcn_readlane((int)(unsigned int)(b & 0xffffffffll), lane);
  int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __builtin_bit_cast(double, (long long)(((unsigned long long)(unsigned int)hi << 32) | (unsigned int)lo));
}
__device__ __forceinline__ int rli(int v, int lane) { return __builtin_amdgcn_readlane(v, lane); }
/* per-lane source (ds_bpermute) */
__device__ __forceinline__ double shf(double v, int src) {
  long long b = __builtin_bit_cast(long long, v);
  int lo = __builtin_amdgcn_ds_bpermute(src << 2, (int)(unsigned int)(b & 0xffffffffll));
  int hi = __builtin_amdgcn_ds_bpermute(src << 2, (int)(b >> 32));
  return __builtin_bit_cast(double, (long long)(((unsigned long long)(unsigned int)hi << 32) | (unsigned int)lo));
}
__device__ __forceinline__ int shfi(int v, int src) { return __builtin_amdgcn_ds_bpermute(src << 2, v); }

/* Constraint rows on the lanes: row r lives on lane r % 64 in slot r / 64 of the lane's RRow array
   (KS::RPL slots: 1 for the compact tier, 2 for the grasp tier).  Lanes whose row is >= nefc have
   typ = -1 and never contribute. */
struct RRow {
  int typ, jj, first; /* jj: row index inside its contact, first: row index of the contact's first row */
  double D, R, aref, floss, mu, fr0, fr1;
  double jar, Jv, force, F; /* the Jacobian row stays in LDS (efc_J): 40 fewer live registers */
  int st, flag;
};

/* the packed mass matrix read with per-row byte bases (1, default) or by KTRI(max, min) (0: A/B) */
#ifndef W_QM_IX
#define W_QM_IX 1
#endif
/* the packed-triangle hand-offs without per-element branches (1, default; see the stores) or with them
   (0: A/B) */
#ifndef W_HL_ORDERED
#define W_HL_ORDERED 1
#endif

/* value of a per-row quantity at row `src` (any slot): a lane shuffle of the slot that holds it.
   With one slot this is the plain shuffle (src 64, 65 wrap to lanes 0, 1 as before; never used). */
template <int RPL>
__device__ __forceinline__ double shfr(const double (&x)[RPL], int src) {
  if constexpr (RPL == 1) {
    return shf(x[0], src);
  } else {
    const double lo = shf(x[0], src & 63), hi = shf(x[1], src & 63);
    return src < 64 ? lo : hi;
  }
}
template <int RPL>
__device__ __forceinline__ int shfri(const int (&x)[RPL], int src) {
  if constexpr (RPL == 1) {
    return shfi(x[0], src);
  } else {
    const int lo = shfi(x[0], src & 63), hi = shfi(x[1], src & 63);
    return src < 64 ? lo : hi;
  }
}

template <class KS>
WD void r_load_rows(KModel m, const KS& s, RRow& w, int r) {
  const int nefc = s.nefc;
  w.typ = -1; w.jj = 0; w.first = r;
  w.D = 0; w.R = 0; w.aref = 0; w.floss = 0; w.mu = 0; w.fr0 = 0; w.fr1 = 0;
  w.jar = 0; w.Jv = 0; w.force = 0; w.F = 0; w.st = ST_SATISFIED; w.flag = 0;
  if (r < nefc) {
    w.typ = s.efc_type[r];
    w.D = s.efc_D[r]; w.R = s.efc_R[r]; w.aref = s.efc_aref[r];
    /* frictionloss rows: efc_id is the dof (r_mc_layout) */
    w.floss = w.typ == CN_FRICTION_DOF ? m->dof_frictionloss[s.efc_id[r]] : 0.0;
    if (w.typ != CN_EQUALITY && w.typ != CN_FRICTION_DOF && w.typ != CN_LIMIT_JOINT) {
      int c = s.efc_id[r];
      int i0 = s.con_efc[c];
      int p = s.con_cpair[c];
      w.first = i0; w.jj = r - i0;
      w.mu = s.con_mu[c];
      w.fr0 = m->cpair_friction[p][0];
      w.fr1 = m->cpair_friction[p][1];
    }
  }
}

/* the constraint Jacobian's unit-vector rows written by readlane, outside the shuffle passes (1, default),
   or every group in the shuffle passes (0: A/B) */
#ifndef W_MC_TRIVIAL
#define W_MC_TRIVIAL 1
#endif
/* the Newton Hessian build skips the first-tree element slot for chunks of quadratic rows without a first-tree
   nonzero (1; their increments there are exactly -0.0) or adds them (0, default): measured 0.5-1 % slower on
   the headline, C3 neutral (profiles/r06_ab A/B 9) */
#ifndef W_T2_SKIP
#define W_T2_SKIP 0
#endif
/* the Newton Hessian's equality-row prefix built once per solve (1, default) or in every direction (0: A/B):
   +1.5 % headline, +1.5-2 % C3 (A/B 9).  Static-tree (main.xml) kernels only: the generic kernel's 8 more
   registers cost it its third wave per SIMD (C2 -2.5 %) */
#ifndef W_HB_EQ_PRE
#define W_HB_EQ_PRE 1
#endif
/* the cone terms' divisions skipped while no contact of the wave is in the cone's middle zone (1,
   default) or always computed (0: A/B) */
#ifndef W_CONE_SKIP
#define W_CONE_SKIP 1
#endif
/* mj_constraintUpdate per row (w_constraint_update) */
template <int RPL>
WD void r_constraint_update(RRow (&W)[RPL]) {
  const int lane = w_lane();
  double jarv[RPL], f0v[RPL], f1v[RPL], f2v[RPL], Fmv[RPL];
  double Nv[RPL], Tv[RPL], U1v[RPL], U2v[RPL];
  int zv[RPL];
  bool anycone = false;
#pragma unroll
  for (int h = 0; h < RPL; h++) jarv[h] = W[h].jar;
#pragma unroll
  for (int h = 0; h < RPL; h++) {
    const RRow& w = W[h];
    const int row = lane + 64 * h;
    const double jar = w.jar;
    /* contact cone: computed on every lane (uniform shuffles), used by contact lanes */
    double jar1 = shfr(jarv, row + 1), jar2 = shfr(jarv, row + 2);
    double mu = w.mu;
    double U0 = jar * mu, U1 = jar1 * w.fr0, U2 = jar2 * w.fr1;
    double N = U0;
    double T2 = 0;
    T2 += U1 * U1;
    T2 += U2 * U2;
    double T = sqrt(T2);
    int z;
    if (N >= mu * T || (T <= 0 && N >= 0)) z = 0;
    else if (mu * N + T <= 0 || (T <= 0 && N < 0)) z = 1;
    else z = 2;
    zv[h] = z;
    Nv[h] = N; Tv[h] = T; U1v[h] = U1; U2v[h] = U2;
    const int t = w.typ;
    anycone |= t >= 0 && t != CN_EQUALITY && t != CN_FRICTION_DOF && t != CN_LIMIT_JOINT && w.jj == 0 && z == 2;
  }
  /* the cone force and cost are read only by the rows of a contact whose first row is in the cone's
     middle zone: with none in the wave (the usual case: sticking or separating contacts), their
     divisions are skipped (the values are then unused, so every result is unchanged) */
  if (!W_CONE_SKIP || w_any<64>(anycone)) {
#pragma unroll
    for (int h = 0; h < RPL; h++) {
      const RRow& w = W[h];
      const double D = w.D, mu = w.mu, N = Nv[h], T = Tv[h], U1 = U1v[h], U2 = U2v[h];
      double Dm = D / (mu * mu * (1 + mu * mu));
      double NT_ = N - mu * T;
      Fmv[h] = 0.5 * Dm * NT_ * NT_;
      f0v[h] = -Dm * NT_ * mu;
      f1v[h] = Dm * NT_ * mu * U1 / T * w.fr0;
      f2v[h] = Dm * NT_ * mu * U2 / T * w.fr1;
    }
  } else {
#pragma unroll
    for (int h = 0; h < RPL; h++) { Fmv[h] = 0.0; f0v[h] = 0.0; f1v[h] = 0.0; f2v[h] = 0.0; }
  }
  /* one code path for every row kind (selects, no per-kind branches): the quadratic terms are formed
     once with the expressions every kind used, the linear friction and cone values beside them */
#pragma unroll
  for (int h = 0; h < RPL; h++) {
    RRow& w = W[h];
    const double jar = w.jar, D = w.D, R = w.R;
    int zs = shfri(zv, w.first);
    double f1s = shfr(f1v, w.first), f2s = shfr(f2v, w.first);
    const int t = w.typ;
    const bool fric = t == CN_FRICTION_DOF;
    const bool contact = t >= 0 && t != CN_EQUALITY && !fric && t != CN_LIMIT_JOINT;
    const double fl = w.floss;
    const bool lneg = fric && jar <= -R * fl;
    const bool lpos = fric && !lneg && jar >= R * fl;
    const bool quad = t == CN_EQUALITY || (fric && !lneg && !lpos) || (t == CN_LIMIT_JOINT && !(jar >= 0)) ||
                      (contact && zs == 1);
    const bool cone = contact && zs != 0 && zs != 1;
    const double qforce = -D * jar, qF = 0.5 * D * jar * jar;
    const double lF0 = -0.5 * R * fl * fl;
    const double lFn = lF0 - fl * jar, lFp = lF0 + fl * jar;
    const int jj = w.jj;
    const double cforce = jj == 0 ? f0v[h] : (jj == 1 ? f1s : f2s);
    w.force = quad ? qforce : (lneg ? fl : (lpos ? -fl : (cone ? cforce : 0.0)));
    w.F = quad ? qF : (lneg ? lFn : (lpos ? lFp : (cone && jj == 0 ? Fmv[h] : w.F)));
    w.flag = (quad || lneg || lpos || (cone && jj == 0)) ? 1 : 0;
    w.st = quad ? ST_QUADRATIC : (lneg ? ST_LINEARNEG : (lpos ? ST_LINEARPOS : (cone ? ST_CONE : ST_SATISFIED)));
  }
}

/* J[row] . x in dof order, the row read from LDS (rows >= nefc: a zero row, as the oracle's
   unused rows never enter a sum; +0 + 0*x stays +0) */
template <class KS>
WD double r_row_dot(const KS& s, int nv, int nefc, const double x[K_NV], int row) {
  const bool act = row < nefc;
  const int r = act ? row : 0;
  /* an inactive row's terms are 0.0 * x[k] = +-0, whose ordered sum from +0 is +0: it returns 0.0
     after the sum instead of selecting 0.0 per element (same value for finite x) */
  double v = 0;
#pragma unroll
  for (int k = 0; k < K_NV; k++)
    if (k < nv) v += s.efc_J[r][k] * x[k];
  return act ? v : 0.0;
}

/* Ordered sums and vector broadcasts inside Newton go through a 64*RPL-double LDS slot per operand
   (with one row slot per lane: the packed-Hessian bytes, unused outside r_direction): each lane
   stores its value(s), then every lane reads the slot in order with broadcast ds_reads, which
   issue back to back, instead of a chain of v_readlane pairs.  Same operands, same order, so the
   sums are unchanged. */
template <class KS>
__device__ __forceinline__ double* r_slot_ptr(KS& s, int k) {
  if constexpr (KS::RPL == 1) return s.Hl + 64 * k;
  else return s.rslot + 64 * KS::RPL * k;
}
#define R_SLOT(s, k) r_slot_ptr(s, k)
WD void r_stage(double* slot, double v) {
  slot[w_lane()] = v;
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}
WD void r_slot_done() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}
/* every row slot of the lanes into `slot` (row r at slot[r]) */
template <int RPL>
WD void r_stage_rows(double* slot, const double (&v)[RPL]) {
#pragma unroll
  for (int h = 0; h < RPL; h++) slot[w_lane() + 64 * h] = v[h];
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

/* ordered sum acc + sl[0] + ... + sl[n-1] over an LDS slot whose entries past n are -0.0 (the exact
   additive identity), so the count rounds up to a multiple of 8 (<= the slot's 64 * RPL entries):
   chunks of 8 reads, the next chunk's reads issued before the current chunk's dependent adds */
WD double r_osum(const double* sl, int n, double acc) {
  const int n8 = (n + 7) & ~7;
  double a[8], b[8];
#pragma unroll
  for (int k = 0; k < 8; k++) a[k] = sl[k];
  for (int i = 0; i < n8;) {
    if (i + 8 < n8) {
#pragma unroll
      for (int k = 0; k < 8; k++) b[k] = sl[i + 8 + k];
    }
#pragma unroll
    for (int k = 0; k < 8; k++) acc += a[k];
    i += 8;
    if (i >= n8) break;
    if (i + 8 < n8) {
#pragma unroll
      for (int k = 0; k < 8; k++) a[k] = sl[i + 8 + k];
    }
#pragma unroll
    for (int k = 0; k < 8; k++) acc += b[k];
    i += 8;
  }
  return acc;
}

/* uniform copy of a dof vector held one element per lane */
WD void r_bcast(double v, int nv, double out[K_NV]) {
#pragma unroll
  for (int k = 0; k < K_NV; k++) out[k] = k < nv ? rl(v, k) : 0.0;
}

/* w_eval_state: Ma (lane k), jar/force/cost terms (per row), gauss and cost (uniform) */
template <class KS>
WD void r_eval_state(KModel m, KS& s, RRow (&W)[KS::RPL], double qacc, double qs, double qas, double& Ma,
                     double& gauss, double& cost) {
  constexpr int RPL = KS::RPL;
  const int lane = w_lane();
  const int nv = NVOF(KS, m), nefc = s.nefc;
  double qv[K_NV];
  r_stage(R_SLOT(s, 0), lane < nv ? qacc : 0.0);
#pragma unroll
  for (int k = 0; k < K_NV; k++) qv[k] = R_SLOT(s, 0)[k];
  {
    double v = 0;
    const int row = lane < nv ? lane : 0;
    const QmIx qi = qm_ix(row);
#pragma unroll
    for (int j = 0; j < K_NV; j++)
      if (j < nv) v += (W_QM_IX ? qm_at(s, qi, j) : qm_get(s, row, j)) * qv[j];
    Ma = v;
  }
#pragma unroll
  for (int h = 0; h < RPL; h++) W[h].jar = r_row_dot(s, nv, nefc, qv, lane + 64 * h) - W[h].aref;
  WT(41);
  r_constraint_update(W);
  WT(42);
  double term = (Ma - qs) * (qacc - qas);
  /* skipped rows contribute -0.0: x + (-0.0) == x exactly for every x (incl. -0, inf, NaN), so
     the ordered sum needs neither a branch nor a select per row */
  double Fm0[RPL], Tm0[RPL];
#pragma unroll
  for (int h = 0; h < RPL; h++) {
    Fm0[h] = W[h].flag ? W[h].F : -0.0;
    Tm0[h] = h == 0 && lane < nv ? term : -0.0;
  }
  double* st = R_SLOT(s, 1);
  double* sf = R_SLOT(s, 2);
#pragma unroll
  for (int h = 0; h < RPL; h++) st[lane + 64 * h] = Tm0[h];
  r_stage_rows(sf, Fm0);
  /* the gauss sum (dofs) on lane 0 and the constraint sum (rows) on lane 1, both over
     max(nv, nefc) entries: the tails are -0.0, so each equals its own ordered sum */
  const int nsum = nv > nefc ? nv : nefc;
  const double* ss = lane == 1 ? sf : st;
  const double acc = r_osum(ss, nsum, 0.0);
  r_slot_done();
  const double a0 = rl(acc, 0), a1 = rl(acc, 1);
  gauss = 0.5 * a0;
  cost = gauss + a1;
  WT(43);
}

/* w_compute_grad: lane k: qfrc_constraint[k] = sum_i J[i][k] force[i] (row order), grad */
template <class KS>
WD void r_compute_grad(KModel m, KS& s, const RRow (&W)[KS::RPL], double Ma, double qs, double& qfrc_c,
                       double& grad) {
  constexpr int RPL = KS::RPL;
  const int lane = w_lane();
  const int nefc = s.nefc;
  const int col = lane < K_NV ? lane : 0;
  double f = 0;
  /* row forces broadcast from an LDS slot; partially unrolled: a fully unrolled MAXEFC-row loop
     hoists every J load at once */
  double* fs = R_SLOT(s, 0);
  double fv[RPL];
#pragma unroll
  for (int h = 0; h < RPL; h++) fv[h] = W[h].force;
  r_stage_rows(fs, fv);
  /* full chunks of 8 rows with the next chunk's J and force reads issued before the current chunk's
     dependent adds, then the remaining rows (row order throughout) */
  const int nfull = nefc & ~7;
  if (nfull > 0) {
    double ja[8], fa[8], jb[8], fb[8];
#pragma unroll
    for (int k = 0; k < 8; k++) { ja[k] = s.efc_J[k][col]; fa[k] = fs[k]; }
    for (int i = 0; i < nfull;) {
      if (i + 8 < nfull) {
#pragma unroll
        for (int k = 0; k < 8; k++) { jb[k] = s.efc_J[i + 8 + k][col]; fb[k] = fs[i + 8 + k]; }
      }
#pragma unroll
      for (int k = 0; k < 8; k++) f = f + ja[k] * fa[k];
      i += 8;
      if (i >= nfull) break;
      if (i + 8 < nfull) {
#pragma unroll
        for (int k = 0; k < 8; k++) { ja[k] = s.efc_J[i + 8 + k][col]; fa[k] = fs[i + 8 + k]; }
      }
#pragma unroll
      for (int k = 0; k < 8; k++) f = f + jb[k] * fb[k];
      i += 8;
    }
  }
#pragma unroll 4
  for (int i = nfull; i < nefc; i++) f = f + s.efc_J[i][col] * fs[i];
  r_slot_done();
  qfrc_c = f;
  grad = Ma - qs - f;
  WT(44);
}

/* compile-time int for generic lambdas */
template <int N>
struct RIc {
  static constexpr int value = N;
};

/* Newton direction: H = M + J'DJ + cone terms (lane k = row k), Cholesky in registers,
   x = H^-1 grad (forward in registers, backward through L^T in LDS); returns -x on lane k */
/* element slots per lane of the Newton Hessian build (K_NV (K_NV + 1) / 2 elements over 64 lanes) */
constexpr int R_NQ = (K_NV * (K_NV + 1) / 2 + 63) / 64;
/* hvp / hvp_ok: the Hessian elements after the equality rows, kept across the directions of one solve */
template <class KS>
WD double r_direction(KModel m, const KPlan* __restrict__ pl, KS& s, const RRow (&W)[KS::RPL], double grad,
                      double (&hvp)[R_NQ], bool& hvp_ok) {
  constexpr int RPL = KS::RPL;
  const int lane = w_lane();
  const int nv = NVOF(KS, m), nefc = s.nefc;
  /* cone Hessians (w_hessian_factor), on each contact's first row */
  {
    double jarv[RPL];
#pragma unroll
    for (int h = 0; h < RPL; h++) jarv[h] = W[h].jar;
#pragma unroll
    for (int h = 0; h < RPL; h++) {
      const RRow& w = W[h];
      const int rowi = lane + 64 * h;
      double jar1 = shfr(jarv, rowi + 1), jar2 = shfr(jarv, rowi + 2);
      if (w.typ >= 0 && w.typ != CN_EQUALITY && w.typ != CN_FRICTION_DOF && w.typ != CN_LIMIT_JOINT &&
          w.jj == 0 && w.st == ST_CONE) {
        int c = s.efc_id[rowi];
        double mu = w.mu;
        double U[3], sc[3];
        sc[0] = mu;
        U[0] = w.jar * mu;
        sc[1] = w.fr0; U[1] = jar1 * sc[1];
        sc[2] = w.fr1; U[2] = jar2 * sc[2];
        double T2 = 0;
        for (int j = 1; j < 3; j++) T2 += U[j] * U[j];
        double T = sqrt(T2);
        double N = U[0];
        double Dm = w.D / (mu * mu * (1 + mu * mu));
        double Hc[3][3];
        Hc[0][0] = 1;
        for (int j = 1; j < 3; j++) {
          Hc[0][j] = -mu * U[j] / T;
          Hc[j][0] = Hc[0][j];
        }
        double muNT = mu * N / T;
        for (int j = 1; j < 3; j++)
          for (int k = 1; k < 3; k++) Hc[j][k] = (j == k ? mu * mu - muNT : 0.0) + muNT * U[j] * U[k] / T2;
        for (int j = 0; j < 3; j++)
          for (int k = 0; k < 3; k++) s.con_Hc[c][3 * j + k] = Hc[j][k] * Dm * sc[j] * sc[k];
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  WT(47);
  const int row = lane < nv ? lane : 0;
  /* H = M + J'DJ + cone blocks in ELEMENT layout: lane owns lower-triangle elements
     e = lane + 64 q (q < 4), each accumulating rows in oracle order; then one LDS transpose
     hands row k to lane k for the factorisation */
  constexpr int NQ = R_NQ;
  /* Block-diagonal case (static tree, s.bdiag: no row couples the two dof trees [0, S) and [S, nv)):
     the oracle's H has exact +0 in the cross block (M has none there, and every J'DJ term it adds
     is a skipped zero or +0 + (+-0) = +0), so its dense Cholesky leaves L's cross block +0 and every
     update a cross entry makes elsewhere subtracts +0 (x - (+0) == x for all x, signed zeros
     included).  Only the two diagonal blocks are then built (126 of 210 elements for main.xml: two
     element slots per lane instead of four) and the factorisation skips the cross updates; the
     triangular solves stay dense. */
  constexpr int SPLIT = KS::STATIC_TREE ? UR3E_MAIN_SPLIT : 0;
  /* the interleaved block Cholesky below runs t < SPLIT and factors the second block's column
     SPLIT + t in step t: it needs the trailing tree to be no larger than the leading one */
  static_assert(UR3E_MAIN_SPLIT == 0 || UR3E_MAIN_NV - UR3E_MAIN_SPLIT <= UR3E_MAIN_SPLIT,
                "block Cholesky: trailing dof tree larger than the leading one");
  const bool bd = SPLIT > 0 && s.bdiag;
#ifdef UR3E_STAGE_TIMING
  if (lane == 0 && bd) s.tcnt[28] += 1; /* diagnostic: block-diagonal Newton directions */
#endif
  const int nel = nv * (nv + 1) / 2;
  const int nel1 = SPLIT * (SPLIT + 1) / 2;
  const int nelb = bd ? nel1 + (nv - SPLIT) * (nv - SPLIT + 1) / 2 : nel;
  const int nqe = (nelb + 63) / 64; /* element slots in use (uniform) */
  auto tri_row = [](int e) {
    int k = (int)((sqrtf(8.0f * (float)e + 1.0f) - 1.0f) * 0.5f);
    while (k * (k + 1) / 2 > e) k--;
    while ((k + 1) * (k + 2) / 2 <= e) k++;
    return k;
  };
  int ek[NQ], ec[NQ], ep[NQ];
  bool ev[NQ];
  double hv[NQ];
#if W_HB_MAP
  static_assert(NQ <= W_HB_NQ, "H element map: more slots than the plan holds");
  {
    /* the lane's element slots from the plan (KPlan.hb_map, the same mapping computed on the host for
       both cases of the block-diagonal flag): one load instead of the triangle-row solve per slot */
    const int* hm = pl->hb_map[(SPLIT > 0 && bd) ? 1 : 0][lane];
#pragma unroll
    for (int q = 0; q < NQ; q++) {
      const int w = hm[q];
      ev[q] = (w >> 24) & 1;
      ek[q] = w & 0xff;
      ec[q] = (w >> 8) & 0xff;
      ep[q] = (w >> 16) & 0xff;
      hv[q] = s.qMp[ep[q]];
    }
  }
#else
#pragma unroll
  for (int q = 0; q < NQ; q++) {
    const int e = lane + 64 * q;
    ev[q] = e < nelb;
    /* second block (bd): local packed index e - nel1, offset by SPLIT; one triangle-row solve either way */
    const bool b2 = bd && e >= nel1;
    const int t = ev[q] ? (b2 ? e - nel1 : e) : 0;
    const int a = tri_row(t);
    const int off = b2 ? SPLIT : 0;
    const int k = off + a, c = off + t - a * (a + 1) / 2;
    ek[q] = ev[q] ? k : 0;
    ec[q] = ev[q] ? c : 0;
    ep[q] = ev[q] ? KTRI(k, c) : 0; /* packed index of element (ek, ec) */
    hv[q] = s.qMp[ep[q]];
  }
#endif
  /* only rows that add to H are visited, in row order (the others add nothing in the oracle):
     quadratic rows and the first row of each cone-state contact; slot h covers rows 64h..
     Rows go in chunks of CH.  Every row's increment is independent of hv: D jk jc for a quadratic
     row (-0.0 where the oracle skips jk == 0: x + (-0.0) == x for every x, signed zeros included),
     the 3x3 cone block for the first row of a cone-state elliptic contact (the only other kind in
     `act`).  So a chunk's loads and products overlap, and only the in-order adds hv += inc stay
     serial: one dependent add per row and element slot.  NQE element slots are compiled in (2 in
     the block-diagonal case, where 126 elements fill two). */
  auto hbuild = [&](auto nqe_tag) {
    constexpr int NQE = decltype(nqe_tag)::value;
    constexpr int CH = NQE <= 2 ? 4 : 2;
    /* block-diagonal element layout (NQE 2): slot 0 holds first-tree elements only (the first block's
       S (S + 1) / 2 >= 64 elements lead), so a chunk of quadratic rows with no first-tree nonzero adds
       exactly -0.0 to every slot-0 element (jk == 0) -- skipped, the same bits (W_T2_SKIP) */
    constexpr bool T2SKIP = W_T2_SKIP && SPLIT > 0 && NQE == 2 && SPLIT * (SPLIT + 1) / 2 >= 64;
#pragma unroll
    for (int h = 0; h < RPL; h++) {
      const RRow& w = W[h];
      const int rb = 64 * h;
      const bool adds = lane + rb < nefc &&
                        (w.st == ST_QUADRATIC || (w.st == ST_CONE && w.typ == CN_CONTACT_ELLIPTIC && w.jj == 0));
      unsigned long long act = __ballot(adds);
      /* rows of this slot that are quadratic with no first-tree nonzero */
      unsigned long long t2q = 0;
#if W_T2_SKIP
      if constexpr (T2SKIP) t2q = s.t2rows[h] & __ballot(lane + rb < nefc && w.st == ST_QUADRATIC);
#endif
      auto run = [&](unsigned long long act) {
      while (act) {
        int r[CH];
        bool v[CH];
        v[0] = true;
        r[0] = (int)__builtin_ctzll(act);
        act &= act - 1;
#pragma unroll
        for (int c = 1; c < CH; c++) { /* past the last row: a repeat of r[0] whose increment is -0.0 */
          v[c] = act != 0;
          r[c] = v[c] ? (int)__builtin_ctzll(act) : r[0];
          act &= act - 1;
        }
        bool skip0 = T2SKIP;
        if constexpr (T2SKIP) {
#pragma unroll
          for (int c = 0; c < CH; c++) skip0 = skip0 && ((t2q >> r[c]) & 1);
        }
        double jk[CH][NQE], jc[CH][NQE];
#pragma unroll
        for (int c = 0; c < CH; c++)
#pragma unroll
          for (int q = 0; q < NQE; q++)
            if (q < nqe && !(q == 0 && skip0)) {
              jk[c][q] = s.efc_J[rb + r[c]][ek[q]];
              jc[c][q] = s.efc_J[rb + r[c]][ec[q]];
            }
        int st[CH];
        double inc[CH][NQE];
#pragma unroll
        for (int c = 0; c < CH; c++) {
          st[c] = rli(w.st, r[c]);
          const double D = rl(w.D, r[c]);
          const bool quad = v[c] && st[c] == ST_QUADRATIC;
#pragma unroll
          for (int q = 0; q < NQE; q++)
            if (q < nqe && !(q == 0 && skip0)) {
              const double djr = D * jk[c][q];
              double t = djr * jc[c][q];
              t = quad && jk[c][q] != 0 ? t : -0.0;
              asm volatile("" : "+v"(t)); /* keeps hv + t from being refolded into a select on hv */
              inc[c][q] = t;
            }
        }
#pragma unroll
        for (int c = 0; c < CH; c++)
          if (v[c] && st[c] != ST_QUADRATIC) {
            const int ri = rb + r[c];
            const double* Hc = s.con_Hc[s.efc_id[ri]];
#pragma unroll
            for (int q = 0; q < NQE; q++) {
              if (q >= nqe) continue;
              double t[3];
              for (int j = 0; j < 3; j++) {
                double acc = 0;
                for (int k = 0; k < 3; k++) acc += Hc[3 * j + k] * s.efc_J[ri + k][ek[q]];
                t[j] = acc;
              }
              double acc = 0;
              for (int j = 0; j < 3; j++) acc += s.efc_J[ri + j][ec[q]] * t[j];
              inc[c][q] = acc;
            }
          }
#pragma unroll
        for (int c = 0; c < CH; c++)
#pragma unroll
          for (int q = 0; q < NQE; q++)
            if (q < nqe && !(q == 0 && skip0)) hv[q] += inc[c][q];
      }
      };
      if constexpr (W_HB_EQ_PRE && KS::STATIC_TREE) {
        if (h == 0) {
          /* the equality rows lead the row order and are always quadratic with fixed D and J, so M plus
             their terms is the same in every Newton direction of this solve: built once (in order, before
             the other rows), then restored (W_HB_EQ_PRE) */
          const unsigned long long eqm = __ballot(lane < nefc && w.typ == CN_EQUALITY);
          if (eqm != 0 && (eqm & (eqm + 1)) == 0) {
            if (hvp_ok) {
#pragma unroll
              for (int q = 0; q < NQE; q++) hv[q] = hvp[q];
            } else {
              run(act & eqm);
#pragma unroll
              for (int q = 0; q < NQE; q++) hvp[q] = hv[q];
              hvp_ok = true;
            }
            act &= ~eqm;
          }
        }
      }
      run(act);
    }
  };
  if constexpr (SPLIT > 0) {
    if (bd) hbuild(RIc<2>{});
    else hbuild(RIc<NQ>{});
  } else {
    hbuild(RIc<NQ>{});
  }
  /* element slot q of this lane is packed-triangle index ep[q] */
#if W_HB_MAP
  if (nelb >= 64) {
    /* every lane's slot 0 is valid and the plan aliases its invalid slots to slot 0's element
       (KPlan.hb_map), so the slots are stored without a per-lane condition, slot 0 last: its valid
       value overwrites the alias (same lane, program order) */
#pragma unroll
    for (int q = NQ - 1; q >= 0; q--)
      if (q < nqe) s.Hl[ep[q]] = hv[q];
  } else
#endif
  {
#pragma unroll
    for (int q = 0; q < NQ; q++)
      if (q < nqe && ev[q]) s.Hl[ep[q]] = hv[q];
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  double h[K_NV];
  /* block-diagonal: the cross block is the oracle's exact +0 (not stored) */
  const int cfrom = bd && row >= SPLIT ? SPLIT : 0;
#pragma unroll
#if W_HL_ORDERED
  for (int c = 0; c < K_NV; c++) { /* unconditional reads, as in the tree factorisation */
    const double v = s.Hl[KTRI(row, c)];
    h[c] = (c <= row && c >= cfrom) ? v : 0.0;
  }
#else
  for (int c = 0; c < K_NV; c++) h[c] = (c <= row && c >= cfrom) ? s.Hl[KTRI(row, c)] : 0.0;
#endif
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  WT(10);
  /* right-looking Cholesky, lane = row; element (i,k) gets -= L[i][j] L[k][j] for j = 0,1,...
     (the oracle's left-looking order) */
  /* L[j][j] ends on lane j (h[j]); the solves read it back by readlane instead of keeping a
     per-lane copy of the whole diagonal */
  if (SPLIT > 0 && bd) {
    /* block-diagonal: the two blocks factor independently (every update of one block by the other
       subtracts +0); their columns are interleaved, column t of the first block with column
       S + t of the second, so the two sqrt / division chains overlap */
    constexpr int NVS = KS::NV;
#pragma unroll
    for (int t = 0; t < SPLIT; t++) {
      const int j = t, jm = SPLIT + t;
      const bool mcol = jm < NVS; /* compile-time (t unrolled) */
      /* one square root and one division per step serve both columns: lanes [0, S) take the first
         block's pivot and entries, lanes [S, ...) the second's (the first block's column on those
         lanes is the cross block's +0, left as it is: +0 / pivot would give +0 again) */
      const bool lb = lane >= SPLIT;
      double sum = rl(h[j], j);
      double summ = mcol ? rl(h[jm < K_NV ? jm : 0], jm < K_NV ? jm : 0) : 1.0;
      double piv = lb ? summ : sum;
      if (piv < K_MINVAL) piv = K_MINVAL;
      const double lp = sqrt(piv); /* lane < S: L[j][j]; lane >= S: L[jm][jm] (1 when !mcol) */
      double& hm = h[jm < K_NV ? jm : 0];
      const double q = (lb ? hm : h[j]) / lp;
      if (!lb && lane > j) h[j] = q;
      if (lane == j) h[j] = lp;
      if (mcol) {
        if (lane > jm) hm = q;
        if (lane == jm) hm = lp;
      }
      double* col = R_SLOT(s, t & 1);
      double* colm = R_SLOT(s, 2);
      col[lane] = h[j];
      if (mcol) colm[lane] = h[jm < K_NV ? jm : 0];
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
      /* every lane updates (no lane >= k select): on lanes < k the entry h[k] is the upper triangle,
         which nothing reads (the diagonal comes from lane k, the solves and the L^T transpose read
         c <= row only) */
#pragma unroll
      for (int k = j + 1; k < SPLIT; k++) {
        const double lkj = col[k];
        h[k] -= h[j] * lkj;
      }
      if (mcol) {
#pragma unroll
        for (int k = jm + 1; k < NVS; k++) {
          const double lkm = colm[k];
          h[k] -= h[jm < K_NV ? jm : 0] * lkm;
        }
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < K_NV; j++) {
      if (j < nv) {
        double sum = rl(h[j], j);
        if (sum < K_MINVAL) sum = K_MINVAL;
        double ljj = sqrt(sum);
        if (lane > j) h[j] = h[j] / ljj;
        if (lane == j) h[j] = ljj;
        /* column j to every lane through an LDS slot (broadcast reads, not a readlane per k) */
        double* col = R_SLOT(s, j & 1);
        r_stage(col, h[j]);
#pragma unroll
        for (int k = j + 1; k < K_NV; k++) {
          if (k < nv) {
            const double lkj = col[k];
            h[k] -= h[j] * lkj; /* upper-triangle entries (lane < k) are never read */
          }
        }
      }
    }
  }
  WT(12);
  /* L^T via LDS (packed lower triangle; the Cholesky's column slots are done with, and nothing else
     reads it during the solves); the diagonal comes back on its own lane */
  if (lane < nv) {
#if W_HL_ORDERED
    /* every lane writes its whole row, c descending, with no per-element branch: a write past the
       diagonal (c > lane) lands on an element (L2, c2) of a later row L2 > lane with c2 < c, which lane
       L2 writes in a later instruction, so the valid value wins (one wave's LDS writes complete in
       order; the compiler barriers keep the program order) */
#pragma unroll
    for (int c = K_NV - 1; c >= 0; c--) {
      s.Hl[KTRI(lane, c)] = h[c];
      asm volatile("" ::: "memory");
    }
#else
#pragma unroll
    for (int c = 0; c < K_NV; c++)
      if (c <= lane) s.Hl[KTRI(lane, c)] = h[c];
#endif
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  /* Both sweeps divide by L[k][k] (>= sqrt(K_MINVAL) > 0).  Lane k divides its own tmp by its own
     pivot and the quotient is read back from lane k: tmp / L[k][k] as k_div_rcp's three operations
     with the pivot's reciprocal taken once (k_div_rcp: correctly rounded, so the same bits as the
     oracle's division) instead of a full division sequence on the uniform operands per step */
  const double dg = lane < nv ? s.Hl[KTRI(row, row)] : 1.0;
  const double rdg = 1.0 / dg;
  /* forward: L y = grad (x[k] = tmp[k] / L[k][k]; tmp[i] -= L[i][k] x[k], i > k).  Every lane applies
     the update (no lane > k select): lane k keeps its result in yf, and the lanes < k, already final in
     yf, only disturb their dead tmp (their h[k] is the unread upper triangle) */
  /* Every lane runs the three operations, but only lane k's quotient is used: the dead lanes' tmp is
     arbitrary, so the numerator check of k_div_rcp would send them to its true division at random.
     Lane k keeps its own numerator (nf), checked once after the sweep; the rare sweep whose used
     numerators left Markstein's range is redone with the true divisions (uniform, same bits). */
  double tmp = grad, yf = 0.0, nf = 0.0;
#pragma unroll
  for (int k = 0; k < K_NV; k++) {
    if (k < nv) {
      double xk = rl(k_div_rcp_raw(tmp, dg, rdg), k);
      yf = lane == k ? xk : yf;
      nf = lane == k ? tmp : nf;
      tmp -= h[k] * xk;
    }
  }
  if (__builtin_expect(w_any<64>(lane < nv && k_rcp_unsafe(nf)), 0)) {
    tmp = grad;
    yf = 0.0;
#pragma unroll
    for (int k = 0; k < K_NV; k++) {
      if (k < nv) {
        const double xk = rl(tmp, k) / rl(dg, k);
        yf = lane == k ? xk : yf;
        tmp -= h[k] * xk;
      }
    }
  }
  WT(18);
  /* lt[i] = L[i][row] for i >= row; for i < row an in-range element nobody uses (KTRI(i, row) <
     nv (nv + 1) / 2 for i < row < nv), so no select */
  double lt[K_NV];
#pragma unroll
  for (int i = 0; i < K_NV; i++) lt[i] = s.Hl[KTRI(i, row)];
  /* backward: L' x = y (x[i] = tmp[i] / L[i][i]; tmp[t] -= L[i][t] x[i], t < i); as the forward sweep,
     every lane updates and lane i keeps x[i] in xf (the lanes > i are final) */
  tmp = yf;
  double xf = 0.0;
  nf = 0.0;
#pragma unroll
  for (int i = K_NV - 1; i >= 0; i--) {
    if (i < nv) {
      double xi = rl(k_div_rcp_raw(tmp, dg, rdg), i); /* lane i: lt[i] = L[i][i] = dg */
      xf = lane == i ? xi : xf;
      nf = lane == i ? tmp : nf;
      tmp -= lt[i] * xi;
    }
  }
  if (__builtin_expect(w_any<64>(lane < nv && k_rcp_unsafe(nf)), 0)) {
    tmp = yf;
    xf = 0.0;
#pragma unroll
    for (int i = K_NV - 1; i >= 0; i--) {
      if (i < nv) {
        const double xi = rl(tmp, i) / rl(dg, i);
        xf = lane == i ? xi : xf;
        tmp -= lt[i] * xi;
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  return -xf;
}

/* line-search 1-D evaluation at a (w_ls_eval): per-row terms on the row lanes, ordered sums */
/* the step-size-independent part of the cone terms, fixed for one line search: the next two rows'
   jar / Jv (lane shuffles) and the V terms (same expressions as before, evaluated once) */
struct RLs {
  double jar1, jar2, Jv1, Jv2, V0, V1, V2, VV, Dm;
};
template <int RPL>
WD void r_ls_setup(const RRow (&W)[RPL], RLs (&C)[RPL]) {
  const int lane = w_lane();
  double jarv[RPL], jvv[RPL];
#pragma unroll
  for (int h = 0; h < RPL; h++) { jarv[h] = W[h].jar; jvv[h] = W[h].Jv; }
#pragma unroll
  for (int h = 0; h < RPL; h++) {
    const RRow& w = W[h];
    RLs& c = C[h];
    const int row = lane + 64 * h;
    c.jar1 = shfr(jarv, row + 1); c.jar2 = shfr(jarv, row + 2);
    c.Jv1 = shfr(jvv, row + 1); c.Jv2 = shfr(jvv, row + 2);
    const double mu = w.mu;
    c.V0 = w.Jv * mu;
    c.V1 = c.Jv1 * w.fr0;
    c.V2 = c.Jv2 * w.fr1;
    c.VV = 0;
    c.VV += c.V1 * c.V1;
    c.VV += c.V2 * c.V2;
    c.Dm = w.D / (mu * mu * (1 + mu * mu));
  }
}

template <class KS>
WD void r_ls_eval(KS& s, const RRow (&W)[KS::RPL], const RLs (&C)[KS::RPL], int nefc, double a, double gauss,
                  double g1, double g2, double& lsF, double& lsdF, double& lsd2F) {
  constexpr int RPL = KS::RPL;
  int zv[RPL];
  double cFv[RPL], cdFv[RPL], cd2Fv[RPL];
  double Nv[RPL], Tv[RPL], T2v[RPL], U1v[RPL], U2v[RPL];
  bool anycone = false;
#pragma unroll
  for (int h = 0; h < RPL; h++) {
    const RRow& w = W[h];
    const RLs& c = C[h];
    /* cone terms from the contact's first row (computed everywhere, used by contact lanes) */
    const double jar1 = c.jar1, jar2 = c.jar2, Jv1 = c.Jv1, Jv2 = c.Jv2;
    double mu = w.mu;
    double U0 = (w.jar + a * w.Jv) * mu;
    double U1 = (jar1 + a * Jv1) * w.fr0;
    double U2 = (jar2 + a * Jv2) * w.fr1;
    double N = U0;
    double T2 = 0;
    T2 += U1 * U1;
    T2 += U2 * U2;
    double T = sqrt(T2);
    int z;
    if (N >= mu * T || (T <= 0 && N >= 0)) z = 0;
    else if (mu * N + T <= 0 || (T <= 0 && N < 0)) z = 1;
    else z = 2;
    zv[h] = z;
    Nv[h] = N; Tv[h] = T; T2v[h] = T2; U1v[h] = U1; U2v[h] = U2;
    const int t = w.typ;
    anycone |= t >= 0 && t != CN_EQUALITY && t != CN_FRICTION_DOF && t != CN_LIMIT_JOINT && w.jj == 0 && z == 2;
  }
  /* the cone terms are read only on the first row of a contact in the middle zone (`cone` below): with
     none in the wave their divisions are skipped (the values are then unused) */
  if (!W_CONE_SKIP || w_any<64>(anycone)) {
#pragma unroll
    for (int h = 0; h < RPL; h++) {
      const RRow& w = W[h];
      const RLs& c = C[h];
      const double mu = w.mu, N = Nv[h], T = Tv[h], T2 = T2v[h], U1 = U1v[h], U2 = U2v[h];
      const double V0 = c.V0, V1 = c.V1, V2 = c.V2;
      const double Dm = c.Dm, VV = c.VV;
      double UV = 0;
      UV += U1 * V1;
      UV += U2 * V2;
      double NT_ = N - mu * T;
      double dNT = V0 - mu * UV / T;
      double d2NT = -mu * (VV * T2 - UV * UV) / (T2 * T);
      cFv[h] = 0.5 * Dm * NT_ * NT_;
      cdFv[h] = Dm * NT_ * dNT;
      cd2Fv[h] = Dm * (dNT * dNT + NT_ * d2NT);
    }
  } else {
#pragma unroll
    for (int h = 0; h < RPL; h++) { cFv[h] = 0.0; cdFv[h] = 0.0; cd2Fv[h] = 0.0; }
  }
  double Fm[RPL], dFm[RPL], d2Fm[RPL];
#pragma unroll
  for (int h = 0; h < RPL; h++) {
    const RRow& w = W[h];
    const double D = w.D, R = w.R;
    double x = w.jar + a * w.Jv;
    double v = w.Jv;
    int zs = shfri(zv, w.first);
    /* one code path for every row kind, as in r_constraint_update */
    const int t = w.typ;
    const bool fric = t == CN_FRICTION_DOF;
    const bool contact = t >= 0 && t != CN_EQUALITY && !fric && t != CN_LIMIT_JOINT;
    const double fl = w.floss;
    const bool lneg = fric && x <= -R * fl;
    const bool lpos = fric && !lneg && x >= R * fl;
    const bool quad = t == CN_EQUALITY || (fric && !lneg && !lpos) || (t == CN_LIMIT_JOINT && x < 0) ||
                      (contact && zs == 1);
    const bool cone = contact && zs == 2 && w.jj == 0;
    const double qF = 0.5 * D * x * x, qdF = D * x * v, qd2F = D * v * v;
    const double lF0 = -0.5 * R * fl * fl;
    const double F = quad ? qF : (lneg ? lF0 - fl * x : (lpos ? lF0 + fl * x : cFv[h]));
    const double dF = quad ? qdF : (lneg ? -fl * v : (lpos ? fl * v : cdFv[h]));
    const double d2F = quad ? qd2F : cd2Fv[h];
    const int flag = (quad || cone) ? 1 : ((lneg || lpos) ? 2 : 0);
    /* skipped terms are -0.0 (exact identity for +), see r_eval_state */
    Fm[h] = flag ? F : -0.0; dFm[h] = flag ? dF : -0.0; d2Fm[h] = flag == 1 ? d2F : -0.0;
  }
  WT(45);
  double aF = gauss + a * g1 + 0.5 * a * a * g2;
  double adF = g1 + a * g2;
  double ad2F = g2;
  double *b0 = R_SLOT(s, 0), *b1 = R_SLOT(s, 1), *b2 = R_SLOT(s, 2);
  const int lane = w_lane();
#pragma unroll
  for (int h = 0; h < RPL; h++) {
    b0[lane + 64 * h] = Fm[h];
    b1[lane + 64 * h] = dFm[h];
  }
  r_stage_rows(b2, d2Fm);
  /* the three ordered sums run on lanes 0, 1, 2 (lane k reads slot k; the others repeat lane 0's):
     one LDS read and one add per row instead of three, same operands in the same order */
  const int sel = lane == 1 ? 1 : (lane == 2 ? 2 : 0);
  const double* bs = R_SLOT(s, sel);
  const double acc = r_osum(bs, nefc, sel == 0 ? aF : (sel == 1 ? adF : ad2F));
  r_slot_done();
  lsF = rl(acc, 0); lsdF = rl(acc, 1); lsd2F = rl(acc, 2);
  WT(46);
}

/* w_line_search: returns alpha (uniform); Jv on the row lanes */
template <class KS>
WD double r_line_search(KModel m, KS& s, RRow (&W)[KS::RPL], double search, double Ma, double qs, double gauss,
                        double scale) {
  constexpr int RPL = KS::RPL;
  const int lane = w_lane();
  const int nv = NVOF(KS, m), nefc = s.nefc;
  double sv[K_NV];
  r_stage(R_SLOT(s, 0), lane < nv ? search : 0.0);
#pragma unroll
  for (int k = 0; k < K_NV; k++) sv[k] = R_SLOT(s, 0)[k];
  r_slot_done();
  double Mv;
  {
    double v = 0;
    const int row = lane < nv ? lane : 0;
    const QmIx qi = qm_ix(row);
#pragma unroll
    for (int j = 0; j < K_NV; j++)
      if (j < nv) v += (W_QM_IX ? qm_at(s, qi, j) : qm_get(s, row, j)) * sv[j];
    Mv = v;
  }
#pragma unroll
  for (int h = 0; h < RPL; h++) W[h].Jv = r_row_dot(s, nv, nefc, sv, lane + 64 * h);
  double t1 = search * (Ma - qs), t2 = search * Mv;
  /* three ordered sums over the dofs on lanes 0, 1, 2 as in r_ls_eval: |search|^2 from the squares
     each lane stages (search_k * search_k, the product every lane formed before), g1, g2 */
  R_SLOT(s, 0)[lane] = search * search;
  R_SLOT(s, 1)[lane] = t1;
  r_stage(R_SLOT(s, 2), t2);
  double gacc = 0;
  {
    const double* gs = R_SLOT(s, lane == 1 ? 1 : (lane == 2 ? 2 : 0));
#pragma unroll
    for (int k = 0; k < K_NV; k++)
      if (k < nv) gacc += gs[k];
  }
  r_slot_done();
  const double snorm = sqrt(rl(gacc, 0));
  if (snorm < K_MINVAL) return 0;
  const double g1 = rl(gacc, 1), g2 = rl(gacc, 2);
  double gtol = m->tolerance * m->ls_tolerance * snorm / scale;
  double f0, d0, h0;
  RLs lc[RPL];
  r_ls_setup(W, lc);
  r_ls_eval(s, W, lc, nefc, 0.0, gauss, g1, g2, f0, d0, h0);
  if (d0 >= 0) return 0;
  double lo = 0.0, dlo = d0, hlo = h0;
  double hi = -1.0, dhi = 0, hhi = 0;
  double bestA = 0.0, bestF = f0;
  double a = -d0 / h0;
  WT(19);
  for (int it = 0; it < m->ls_iterations; it++) {
    double f, df, d2f;
    r_ls_eval(s, W, lc, nefc, a, gauss, g1, g2, f, df, d2f);
    WT(20);
    if (f < bestF) { bestF = f; bestA = a; }
    if (fabs(df) < gtol) return (f <= bestF) ? a : bestA;
    if (df < 0) { lo = a; dlo = df; hlo = d2f; }
    else { hi = a; dhi = df; hhi = d2f; }
    double na;
    if (hi < 0) {
      na = a - df / d2f;
      if (!(na > a)) na = 2 * a;
    } else {
      double c1 = lo - dlo / hlo;
      double c2 = hi - dhi / hhi;
      if (c1 > lo && c1 < hi) na = c1;
      else if (c2 > lo && c2 < hi) na = c2;
      else na = 0.5 * (lo + hi);
    }
    a = na;
  }
  return bestA;
}

/* diagnostic builds only (-DUR3E_DOUBLE_STAGE=20..23): run one Newton component twice (direction,
   line search, constraint-state evaluation, gradient; each idempotent) for tools/stage_insts.py */
#ifndef UR3E_DOUBLE_STAGE
#define UR3E_DOUBLE_STAGE -1
#endif
#define RDBL(k, stmt) do { stmt; if (UR3E_DOUBLE_STAGE == (k)) { stmt; } } while (0)
/* w_solve_newton for the compact tier; leaves s.qacc and s.qfrc_constraint */
template <class KS>
WD void r_solve_newton(KModel m, const KPlan* __restrict__ pl, KS& s) {
  constexpr int RPL = KS::RPL;
  const int lane = w_lane();
  const int nv = NVOF(KS, m);
  if (s.nefc == 0) {
    if (lane < nv) { s.qacc[lane] = s.qacc_smooth[lane]; s.qfrc_constraint[lane] = 0; }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    return;
  }
  const double scale = 1.0 / (m->meaninertia * (nv > 1 ? nv : 1));
  const int k = lane < nv ? lane : 0;
  const double qs = s.qfrc_smooth[k], qas = s.qacc_smooth[k];
  double qacc = lane < nv ? s.warm[k] : 0.0;
  RRow W[RPL];
#pragma unroll
  for (int h = 0; h < RPL; h++) r_load_rows(m, s, W[h], lane + 64 * h);
  /* the rows' R / D / aref share bytes with Hl and the ordered-sum slots (W_ROWS_IN_HL): read before any
     of those is written */
#ifndef W_LOAD_FENCE
#define W_LOAD_FENCE 1
#endif
  if (W_LOAD_FENCE && KS::RHL) {
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
  }
  double Ma, gauss, cost;
  RDBL(22, r_eval_state(m, s, W, qacc, qs, qas, Ma, gauss, cost));
  const double cost_ws = cost;
  /* the warm start's evaluation is kept: when it wins, the oracle evaluates it again, and that
     deterministic recomputation (same qacc, same rows) is replaced by restoring what it produces
     (jar, force, F, state, flag per row; Ma, gauss, cost) */
  double k_jar[RPL], k_force[RPL], k_F[RPL];
  int k_st[RPL], k_flag[RPL];
#pragma unroll
  for (int h = 0; h < RPL; h++) {
    k_jar[h] = W[h].jar; k_force[h] = W[h].force; k_F[h] = W[h].F; k_st[h] = W[h].st; k_flag[h] = W[h].flag;
  }
  const double k_Ma = Ma, k_gauss = gauss;
  RDBL(22, r_eval_state(m, s, W, lane < nv ? qas : 0.0, qs, qas, Ma, gauss, cost));
  const double cost_sm = cost;
  if (cost_ws > cost_sm) {
    qacc = lane < nv ? qas : 0.0;
  } else {
#pragma unroll
    for (int h = 0; h < RPL; h++) {
      W[h].jar = k_jar[h]; W[h].force = k_force[h]; W[h].F = k_F[h]; W[h].st = k_st[h]; W[h].flag = k_flag[h];
    }
    Ma = k_Ma; gauss = k_gauss; cost = cost_ws;
  }
  double qfrc_c, grad;
  RDBL(23, r_compute_grad(m, s, W, Ma, qs, qfrc_c, grad));
  WT(9);
  double search;
  double hvp[R_NQ];
  bool hvp_ok = false;
  RDBL(20, search = r_direction(m, pl, s, W, grad, hvp, hvp_ok));
  WT(11);
  for (int iter = 0; iter < m->iterations; iter++) {
    double alpha;
    RDBL(21, alpha = r_line_search(m, s, W, search, Ma, qs, gauss, scale));
    WT(13);
    if (alpha == 0) break;
    qacc += alpha * search;
    double oldcost = cost;
    RDBL(22, r_eval_state(m, s, W, qacc, qs, qas, Ma, gauss, cost));
    RDBL(23, r_compute_grad(m, s, W, Ma, qs, qfrc_c, grad));
    WT(14);
    /* lane i stages grad_i * grad_i (the product every lane formed before), then one ordered sum */
    double gn = 0;
    r_stage(R_SLOT(s, 0), grad * grad);
#pragma unroll
    for (int i = 0; i < K_NV; i++)
      if (i < nv) gn += R_SLOT(s, 0)[i];
    r_slot_done();
    double improvement = scale * (oldcost - cost);
    double gradient = scale * sqrt(gn);
    if (improvement < m->tolerance || gradient < m->tolerance) break;
    RDBL(20, search = r_direction(m, pl, s, W, grad, hvp, hvp_ok));
    WT(11);
  }
  if (lane < nv) { s.qacc[lane] = qacc; s.qfrc_constraint[lane] = qfrc_c; }
  /* touch sensors read the contact normal forces */
#pragma unroll
  for (int h = 0; h < RPL; h++)
    if (lane + 64 * h < s.nefc) s.efc_force[lane + 64 * h] = W[h].force;
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

/* mj_factorI + mj_solveLD on A = qM (+ h*damping on the diagonal when `damped`), compact tier:
   the reverse tree LDL' runs in registers in COLUMN layout (lane j holds A[i][j] for all i), so
   every cross-lane operand is a readlane of a constant register index; the forward substitution
   needs rows and gets them through one LDS transpose (s.H).  Same element update order as
   w_factor_tree / w_solve_tree.  Returns x = A^-1 b on lane t (< nv). */
template <class KS>
WD double r_tree_solve(KModel m, const KPlan* __restrict__ pl, KS& s, bool damped, double b) {
  const int lane = w_lane();
  const int nv = NVOF(KS, m);
  const int col = lane < nv ? lane : 0;
  /* plan masks and damping up front: one batch of scalar loads, not one wait per column */
  unsigned int amask[K_NV];
#pragma unroll
  for (int k = 0; k < K_NV; k++)
    amask[k] = KS::STATIC_TREE ? (k < UR3E_MAIN_NV ? ur3e_main_dof_anc_mask[k] : 0u) : pl->dof_anc_mask[k];
  double a[K_NV];
  {
    const QmIx qc = qm_ix(col); /* M[i][col] = M[col][i]: the same packed element */
#pragma unroll
    for (int i = 0; i < K_NV; i++) a[i] = W_QM_IX ? qm_at(s, qc, i) : qm_get(s, i, col);
  }
  if (damped) {
    const double hstep = m->timestep;
    const double dmp = lane < nv ? m->dof_damping[col] : 0.0;
    const double add = hstep * dmp;
#pragma unroll
    for (int i = 0; i < K_NV; i++)
      if (lane == i && i < nv) a[i] += add;
  }
  const unsigned int lbit = lane < 32 ? (1u << lane) : 0u;
  /* main.xml: the dofs split into two trees [0, S) and [S, nv) with no ancestor across (the arm with
     the gripper, the mug's free joint), so no element of one tree is ever updated by a pivot of the
     other.  Their pivots are paired, S - 1 - t with nv - 1 - t in step t: one division, one staged
     multiplier slot (lanes [0, S) carry the first tree's, lanes [S, nv) the second's) and both
     update sets per step, so the two pivot chains overlap.  Every element still gets its updates in
     the oracle's (descending pivot) order: bit-identical. */
  constexpr int SPLIT = KS::STATIC_TREE ? UR3E_MAIN_SPLIT : 0;
  if constexpr (SPLIT > 0) {
    constexpr int NVS = KS::NV;
    static_assert(NVS - SPLIT <= SPLIT, "paired tree LDL': trailing dof tree larger than the leading one");
    const bool lb = lane >= SPLIT;
#pragma unroll
    for (int t = 0; t < SPLIT; t++) {
      const int ka = SPLIT - 1 - t, km0 = NVS - 1 - t;
      const bool mcol = km0 >= SPLIT; /* compile-time (t unrolled) */
      const int km = mcol ? km0 : 0;
      double akka = rl(a[ka], ka);
      if (akka < K_MINVAL) akka = K_MINVAL;
      double akkm = mcol ? rl(a[km], km) : 1.0;
      if (akkm < K_MINVAL) akkm = K_MINVAL;
      if (lane == ka) a[ka] = akka;
      if (mcol && lane == km) a[km] = akkm;
      const unsigned int ama = amask[ka], amm = mcol ? amask[km] : 0u;
      if (ama | amm) {
        const double tmp = (lb ? a[km] : a[ka]) / (lb ? akkm : akka);
        double* tk = R_SLOT(s, t & 1);
        r_stage(tk, tmp);
        /* every lane updates, without the lane-in-anc(k) and lane <= i masks: a lane outside them
           holds, in row i, an element no later step reads (upper triangle, or a column that is not
           an ancestor of row i: the factor, the sweeps and the transpose below only read ancestor
           pairs and the diagonal) */
#pragma unroll
        for (int i = 0; i < ka; i++) {
          if ((ama >> i) & 1u) {
            const double ti = tk[i];
            a[i] -= a[ka] * ti;
          }
        }
#pragma unroll
        for (int i = SPLIT; i < km; i++) {
          if ((amm >> i) & 1u) {
            const double ti = tk[i];
            a[i] -= a[km] * ti;
          }
        }
        if (ama & lbit) a[ka] = tmp;
        if (amm & lbit) a[km] = tmp;
      }
    }
  } else {
#pragma unroll
    for (int k = K_NV - 1; k >= 0; k--) {
      if (k < nv) {
        double akk = rl(a[k], k);
        if (akk < K_MINVAL) akk = K_MINVAL;
        if (lane == k) a[k] = akk;
        const unsigned int am = amask[k];
        if (am) {
          double tmp = a[k] / akk; /* lane i in anc(k): A[k][i] / A[k][k] */
          /* the multipliers reach every lane through an LDS slot (broadcast reads) */
          double* tk = R_SLOT(s, k & 1);
          r_stage(tk, tmp);
#pragma unroll
          for (int i = 0; i < k; i++) {
            if ((am >> i) & 1u) {
              const double ti = tk[i];
              if ((am & lbit) && lane <= i) a[i] -= a[k] * ti;
            }
          }
          if (am & lbit) a[k] = tmp;
        }
      }
    }
  }
  WT(40);
  double dg = 1.0;
#pragma unroll
  for (int i = 0; i < K_NV; i++)
    if (lane == i && i < nv) dg = a[i];
  const double dinv = 1.0 / dg;
  double x = lane < nv ? b : 0.0;
  if constexpr (SPLIT > 0) {
    /* the same pairing: x_i's updates come from its tree's descendants only, in descending order */
    constexpr int NVS = KS::NV;
#pragma unroll
    for (int t = 0; t < SPLIT; t++) {
      const int ia = SPLIT - 1 - t, im0 = NVS - 1 - t;
      const bool mcol = im0 >= SPLIT;
      const int im = mcol ? im0 : 0;
      const unsigned int ama = amask[ia], amm = mcol ? amask[im] : 0u;
      if (ama | amm) {
        const double xa = rl(x, ia);
        const double xm = mcol ? rl(x, im) : 0.0;
        const bool ua = (ama & lbit) != 0, um = (amm & lbit) != 0;
        const double prod = ua ? a[ia] * xa : a[im] * xm;
        if (ua || um) x -= prod;
      }
    }
  } else {
#pragma unroll
    for (int i = K_NV - 1; i >= 0; i--) {
      if (i < nv) {
        const unsigned int am = amask[i];
        if (am) {
          double xi = rl(x, i);
          if (am & lbit) x -= a[i] * xi;
        }
      }
    }
  }
  if (lane < nv) x *= dinv;
  /* column -> row hand-off through the packed lower triangle (ancestors have lower indices) */
  if (lane < nv) {
#if W_HL_ORDERED
    /* every lane writes its whole column, i ascending, with no per-element branch: a write above the
       diagonal (i < lane) lands on an element (i2, c2) of a later row i2 > i, written in a later
       instruction, so the valid value wins (as in the Newton direction's L' hand-off) */
#pragma unroll
    for (int i = 0; i < K_NV; i++) {
      s.Hl[KTRI(i, lane)] = a[i];
      asm volatile("" ::: "memory");
    }
#else
#pragma unroll
    for (int i = 0; i < K_NV; i++)
      if (i >= lane) s.Hl[KTRI(i, lane)] = a[i];
#endif
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  const unsigned int myam = lane < nv ? pl->dof_anc_mask[lane] : 0u;
  double r[K_NV];
#pragma unroll
#if W_HL_ORDERED
  /* unconditional reads (KTRI(col, j) < K_NV (K_NV + 1) / 2 for every j): no per-element branch */
  for (int j = 0; j < K_NV; j++) {
    const double v = s.Hl[KTRI(col, j)];
    r[j] = j <= col ? v : 0.0;
  }
#else
  for (int j = 0; j < K_NV; j++) r[j] = j <= col ? s.Hl[KTRI(col, j)] : 0.0;
#endif
  if constexpr (SPLIT > 0) {
    /* paired again: ancestor j of a lane is in the lane's own tree, ascending within it */
    constexpr int NVS = KS::NV;
    const bool lb = lane >= SPLIT;
#pragma unroll
    for (int t = 0; t < SPLIT; t++) {
      const int ja = t, jm0 = SPLIT + t;
      const bool mcol = jm0 < NVS;
      const int jm = mcol ? jm0 : 0;
      const double xa = rl(x, ja);
      const double xm = mcol ? rl(x, jm) : 0.0;
      const bool ua = !lb && ((myam >> ja) & 1u), um = mcol && lb && ((myam >> jm) & 1u);
      const double prod = ua ? r[ja] * xa : r[jm] * xm;
      if (ua || um) x -= prod;
    }
  } else {
#pragma unroll
    for (int j = 0; j < K_NV; j++) {
      if (j < nv) {
        double xj = rl(x, j);
        if ((myam >> j) & 1u) x -= r[j] * xj;
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  return x;
}

/* subtree accumulation f[parent(i)] += f[i] for i = nbody-1 .. 1 (the oracle's order), lane = body,
   as a readlane chain in registers instead of read-modify-write round trips through LDS;
   SKIP_WORLD leaves body 0 out (crb) */
template <int C, bool SKIP_WORLD>
WD void r_subtree_sum(KModel m, double (&f)[C]) {
  const int lane = w_lane();
  const int nb = m->nbody;
  int par[K_NB];
#pragma unroll
  for (int i = 0; i < K_NB; i++) par[i] = i < nb ? m->body_parentid[i] : 0;
#pragma unroll
  for (int i = K_NB - 1; i > 0; i--) {
    if (i < nb) {
      const int p = par[i];
      if (!SKIP_WORLD || p > 0) {
        double v[C];
#pragma unroll
        for (int c = 0; c < C; c++) v[c] = rl(f[c], i);
        if (lane == p) {
#pragma unroll
          for (int c = 0; c < C; c++) f[c] += v[c];
        }
      }
    }
  }
}

/* main.xml (static body tree): the same subtree sums with the components across lanes.  Lane c < C
   reads component c of every body from the LDS rows src[i][c] into registers, adds child into parent
   for i = nb-1 .. 1 (the oracle's order; the parents are compile-time, so the adds are register to
   register and only the tree's own dependencies order them) and writes the sums to dst[i][c] (src
   and dst may be the same rows).  One pass of loads and stores instead of 20-24 readlane steps of C
   doubles each.  The caller has made src visible (wave barrier); dst is visible on return. */
template <int C, bool SKIP_WORLD, int SS, int DS>
WD void r_subtree_sum_cols(const double (*src)[SS], double (*dst)[DS]) {
  static_assert(C <= SS && C <= DS, "subtree sum: component count exceeds the row");
  const int lane = w_lane();
  if (lane < C) {
    double F[UR3E_MAIN_NB];
#pragma unroll
    for (int i = 0; i < UR3E_MAIN_NB; i++) F[i] = src[i][lane];
#pragma unroll
    for (int i = UR3E_MAIN_NB - 1; i > 0; i--) {
      const int p = ur3e_main_body_parent[i];
      if (!SKIP_WORLD || p > 0) F[p] += F[i];
    }
#pragma unroll
    for (int i = 0; i < UR3E_MAIN_NB; i++) dst[i][lane] = F[i];
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

/* ================================================================== */
/* body-tree passes for the compact tier (lane = body, nbody <= 64)    */
/* ================================================================== */
/* every per-body model constant a pass needs is loaded before its level loop, so a level
   costs one LDS read of the parent + the arithmetic, not a chain of dependent global loads;
   bodies carry at most one joint (KPlan.max_jntnum <= 1, checked by the caller) */

/* w_kinematics (mj_kinematics) */
template <class KS>
WD void r_kinematics(KModel m, const KPlan* __restrict__ pl, KS& s) {
  const int lane = w_lane();
  const int nb = m->nbody, nlevel = pl->nlevel;
  const int b = lane < nb ? lane : 0;
  const int depth = (lane < nb && lane > 0) ? pl->body_depth[b] : -1;
  const int pid = m->body_parentid[b];
  const int jn = m->body_jntnum[b];
  const int jf = m->body_jntadr[b];
  /* the body's joint constants flattened per body in the plan: one load level */
  const int jt = pl->bj_type[b];
  const int qa = pl->bj_qadr[b];
  double bpos[3], bquat[4], jax[3], jps[3];
  for (int c = 0; c < 3; c++) { bpos[c] = m->body_pos[b][c]; jax[c] = pl->bj_axis[b][c]; jps[c] = pl->bj_pos[b][c]; }
  for (int c = 0; c < 4; c++) bquat[c] = m->body_quat[b][c];
  const double q0 = pl->bj_q0[b];
  /* frames hanging off bodies: lane g < ngeom -> geom g, then sites */
  const int ng = m->ngeom, nfr = m->ngeom + m->nsite;
  int fb = 0;
  double fpos[3] = {0, 0, 0}, fquat[4] = {1, 0, 0, 0};
  if (W_FLAT_DYN) {
    /* geoms then sites, one plan row each (KPlan.fr_*): one branch and one load level */
    if (lane < nfr) {
      fb = pl->fr_b[lane];
      for (int c = 0; c < 3; c++) fpos[c] = pl->fr_d[lane][c];
      for (int c = 0; c < 4; c++) fquat[c] = pl->fr_d[lane][3 + c];
    }
  } else if (lane < ng) {
    fb = m->geom_bodyid[lane];
    for (int c = 0; c < 3; c++) fpos[c] = m->geom_pos[lane][c];
    for (int c = 0; c < 4; c++) fquat[c] = m->geom_quat[lane][c];
  } else if (lane < nfr) {
    const int q = lane - ng;
    fb = m->site_bodyid[q];
    for (int c = 0; c < 3; c++) fpos[c] = m->site_pos[q][c];
    for (int c = 0; c < 4; c++) fquat[c] = m->site_quat[q][c];
  }
  /* hinge rotation of this body's joint (w_kinematics' qloc pass) */
  double ql[4] = {1, 0, 0, 0};
  if (depth > 0 && jn == 1 && jt != UR3E_JNT_FREE) k_axis_angle_quat(ql, jax, s.qpos[qa] - q0);
  if (lane == 0) {
    s.xpos[0][0] = s.xpos[0][1] = s.xpos[0][2] = 0;
    s.xquat[0][0] = 1; s.xquat[0][1] = s.xquat[0][2] = s.xquat[0][3] = 0;
    k_quat2mat(s.xmat[0], s.xquat[0]);
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  /* MuJoCo's per-body recurrence (mj_kinematics), split so that only its true dependency chain runs
     level by level:
       1. orientation chain: q1 = parent xquat * body_quat, q2 = q1 * qloc, xquat = normalize(q2);
       2. every body at once: xmat = quat2mat(xquat), the joint axis and the two joint-position
          rotations (by q1 and by q2), and tv = parent xmat * body_pos;
       3. position chain: xpos = ((parent xpos + tv) + xanchor offset) - rotated joint pos.
     Every value is the same expression of the same operands as in the one-pass recurrence (only
     its place in time moves), so the results are bit-identical; the 13-level chain now carries
     ~100 instructions per level instead of ~550. */
  const bool isfree = jn == 1 && jt == UR3E_JNT_FREE;
  const bool hinge = depth > 0 && jn == 1 && !isfree;
  double q1[4] = {1, 0, 0, 0}, q2[4] = {1, 0, 0, 0}, xq[4] = {1, 0, 0, 0};
  for (int lvl = 1; lvl <= nlevel; lvl++) {
    if (depth == lvl) {
      if (isfree) {
        xq[0] = s.qpos[qa + 3]; xq[1] = s.qpos[qa + 4]; xq[2] = s.qpos[qa + 5]; xq[3] = s.qpos[qa + 6];
      } else {
        double pq[4];
        for (int c = 0; c < 4; c++) pq[c] = s.xquat[pid][c];
        k_mul_quat(q1, pq, bquat);
        if (jn == 1) k_mul_quat(q2, q1, ql);
        else for (int c = 0; c < 4; c++) q2[c] = q1[c];
        for (int c = 0; c < 4; c++) xq[c] = q2[c];
      }
      k_normalize4(xq);
      for (int c = 0; c < 4; c++) s.xquat[lane][c] = xq[c];
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
  }
  WT(29);
  /* 2. orientation-only terms of every body */
  double ra[3] = {0, 0, 0}, vec[3] = {0, 0, 0};
  if (depth > 0) {
    double xm[9];
    k_quat2mat(xm, xq);
    for (int c = 0; c < 9; c++) s.xmat[lane][c] = xm[c];
    if (hinge) {
      double xaxis[3];
      k_rot_vec_quat(xaxis, jax, q1);
      k_rot_vec_quat(ra, jps, q1);
      k_rot_vec_quat(vec, jps, q2);
      for (int c = 0; c < 3; c++) s.xaxis[jf][c] = xaxis[c];
    } else if (isfree) {
      s.xaxis[jf][0] = 0; s.xaxis[jf][1] = 0; s.xaxis[jf][2] = 1;
    }
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  double tv[3] = {0, 0, 0};
  if (depth > 0 && !isfree) {
    double pm[9];
    for (int c = 0; c < 9; c++) pm[c] = s.xmat[pid][c];
    k_mat_vec3(tv, pm, bpos);
  }
  /* 3. position chain */
  if constexpr (KS::STATIC_TREE && UR3E_MAIN_BODY_COLS) {
    /* main.xml: with the components across lanes.  Each body stages its terms -- tv in its xpos row,
       ra in its joint's xanchor row, vec in its joint's qloc row (unused by this path); a free body
       (a child of the world) its final position -- then lane c < 3 walks the bodies in index order
       in registers: P = parent + tv, and for a hinge anchor = ra + P, P = anchor - vec. */
    if (depth > 0) {
      if (isfree) {
        for (int c = 0; c < 3; c++) { s.xpos[lane][c] = s.qpos[qa + c]; s.xanchor[jf][c] = s.qpos[qa + c]; }
      } else {
        for (int c = 0; c < 3; c++) s.xpos[lane][c] = tv[c];
        if (jn == 1)
          for (int c = 0; c < 3; c++) { s.xanchor[jf][c] = ra[c]; s.qloc[jf][c] = vec[c]; }
      }
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    if (lane < 3) {
      double P[UR3E_MAIN_NB];
#pragma unroll
      for (int i = 0; i < UR3E_MAIN_NB; i++) P[i] = s.xpos[i][lane];
#pragma unroll
      for (int i = 1; i < UR3E_MAIN_NB; i++) {
        const int p = ur3e_main_body_parent[i], dn = ur3e_main_body_dofnum[i], j = ur3e_main_body_jntadr[i];
        if (dn == 0) {
          P[i] = P[p] + P[i];
        } else if (dn == 1) {
          const double xa = s.xanchor[j][lane] + (P[p] + P[i]);
          P[i] = xa - s.qloc[j][lane];
          s.xanchor[j][lane] = xa;
        }
      }
#pragma unroll
      for (int i = 1; i < UR3E_MAIN_NB; i++) s.xpos[i][lane] = P[i];
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
  } else {
    for (int lvl = 1; lvl <= nlevel; lvl++) {
      if (depth == lvl) {
        double xpos[3];
        if (isfree) {
          xpos[0] = s.qpos[qa]; xpos[1] = s.qpos[qa + 1]; xpos[2] = s.qpos[qa + 2];
          s.xanchor[jf][0] = xpos[0]; s.xanchor[jf][1] = xpos[1]; s.xanchor[jf][2] = xpos[2];
        } else {
          for (int c = 0; c < 3; c++) xpos[c] = s.xpos[pid][c] + tv[c];
          if (jn == 1) {
            double xanchor[3];
            for (int c = 0; c < 3; c++) xanchor[c] = ra[c] + xpos[c];
            for (int c = 0; c < 3; c++) xpos[c] = xanchor[c] - vec[c];
            for (int c = 0; c < 3; c++) s.xanchor[jf][c] = xanchor[c];
          }
        }
        for (int c = 0; c < 3; c++) s.xpos[lane][c] = xpos[c];
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
    }
  }
  WT(30);
  if (lane < nfr) {
    double bp[3], bq[4], bm[9], op[3], om[9];
    for (int c = 0; c < 3; c++) bp[c] = s.xpos[fb][c];
    for (int c = 0; c < 4; c++) bq[c] = s.xquat[fb][c];
    for (int c = 0; c < 9; c++) bm[c] = s.xmat[fb][c];
    k_local2global(op, om, bp, bq, bm, fpos, fquat);
    if (lane < ng) {
      for (int c = 0; c < 3; c++) s.geom_xpos[lane][c] = op[c];
      for (int c = 0; c < 9; c++) s.geom_xmat[lane][c] = om[c];
    } else {
      for (int c = 0; c < 3; c++) s.site_xpos[lane - ng][c] = op[c];
      for (int c = 0; c < 9; c++) s.site_xmat[lane - ng][c] = om[c];
    }
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

/* main.xml (static body tree): a root-to-leaf chain over the rows of a [body][6+] array with the six
   components across lanes.  Row i holds body i's staged increment; lane c < 6 walks the bodies in
   index order (parents first) in registers: ALL == false (velocities): V[i] = V[p] for a body
   without dofs, V[p] + row[i] for a one-dof body, row[i] as staged for a several-dof body (a child
   of the world, computed on its lane); ALL == true (accelerations): V[i] = V[p] + row[i] for every
   body.  Row 0 (the world) is the start value.  The rows are overwritten with V. */
template <bool ALL, int DS>
WD void r_chain_cols(double (*rows)[DS]) {
  const int lane = w_lane();
  if (lane < 6) {
    double V[UR3E_MAIN_NB];
#pragma unroll
    for (int i = 0; i < UR3E_MAIN_NB; i++) V[i] = rows[i][lane];
#pragma unroll
    for (int i = 1; i < UR3E_MAIN_NB; i++) {
      const int p = ur3e_main_body_parent[i], dn = ur3e_main_body_dofnum[i];
      if (ALL || dn == 1) V[i] = V[p] + V[i];
      else if (dn == 0) V[i] = V[p];
    }
#pragma unroll
    for (int i = 1; i < UR3E_MAIN_NB; i++) rows[i][lane] = V[i];
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

/* w_com_vel fused with the forward (cacc) pass of w_rne_passive: both only need the parent's
   values, so one level sweep produces cvel, cdof_dot and cacc */
template <class KS>
WD void r_vel_acc(KModel m, const KPlan* __restrict__ pl, KS& s) {
  const int lane = w_lane();
  const int nb = m->nbody, nlevel = pl->nlevel;
  const int b = lane < nb ? lane : 0;
  const int depth = (lane < nb && lane > 0) ? pl->body_depth[b] : -1;
  const int pid = m->body_parentid[b];
  const int bda = m->body_dofadr[b];
  const int bdn = m->body_dofnum[b];
  /* one joint per body on this path's models: the first dof's joint is the body's first joint */
  const bool onejnt = KS::STATIC_TREE || pl->max_jntnum <= 1;
  const int jt = bdn ? (onejnt ? pl->bj_type[b] : m->jnt_type[m->dof_jntid[bda]]) : UR3E_JNT_HINGE;
  auto cacc = w_cacc(s);
  auto cdof_dot = w_cdof_dot(s);
  /* single-dof bodies: their cdof row and qvel, loaded up front */
  double cd[6] = {0, 0, 0, 0, 0, 0}, qv = 0;
  if (bdn == 1) {
    for (int r = 0; r < 6; r++) cd[r] = s.cdof[bda][r];
    qv = s.qvel[bda];
  }
  if (lane == 0) {
    for (int k = 0; k < 6; k++) s.cvel[0][k] = 0;
    cacc[0][0] = cacc[0][1] = cacc[0][2] = 0;
    cacc[0][3] = -m->gravity[0]; cacc[0][4] = -m->gravity[1]; cacc[0][5] = -m->gravity[2];
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  /* Split like r_kinematics: the velocity chain cvel = parent cvel + cdof * qvel runs level by level,
     then cdof_dot and the acceleration term of every single-dof body are formed at once, then the
     chain cacc = parent cacc + term.  Same expressions, same operands: bit-identical. */
  const bool one = bdn == 1 && jt != UR3E_JNT_FREE;
  double cqv[6], cvp[6] = {0, 0, 0, 0, 0, 0}, tmp[6] = {0, 0, 0, 0, 0, 0};
  for (int r = 0; r < 6; r++) cqv[r] = cd[r] * qv;
  /* general body (free joint, several dofs, none): w_com_vel on cv (the parent's cvel), and its cacc
     term in tmp */
  auto general = [&](double (&cv)[6]) {
    for (int j = 0; j < bdn; j++) {
      int dof = bda + j;
      int jtj = onejnt ? jt : m->jnt_type[m->dof_jntid[dof]];
      if (jtj == UR3E_JNT_FREE) {
        for (int k = 0; k < 3; k++)
          for (int r = 0; r < 6; r++) cdof_dot[dof + k][r] = 0;
        double tq[6] = {0, 0, 0, 0, 0, 0};
        for (int k = 0; k < 3; k++)
          for (int r = 0; r < 6; r++) tq[r] += s.cdof[dof + k][r] * s.qvel[dof + k];
        for (int r = 0; r < 6; r++) cv[r] += tq[r];
        for (int k = 3; k < 6; k++) k_cross_motion(cdof_dot[dof + k], cv, s.cdof[dof + k]);
        for (int r = 0; r < 6; r++) tq[r] = 0;
        for (int k = 3; k < 6; k++)
          for (int r = 0; r < 6; r++) tq[r] += s.cdof[dof + k][r] * s.qvel[dof + k];
        for (int r = 0; r < 6; r++) cv[r] += tq[r];
        j += 5;
      } else {
        k_cross_motion(cdof_dot[dof], cv, s.cdof[dof]);
        for (int r = 0; r < 6; r++) cv[r] += s.cdof[dof][r] * s.qvel[dof];
      }
    }
    for (int j = 0; j < bdn; j++)
      for (int r = 0; r < 6; r++) tmp[r] += cdof_dot[bda + j][r] * s.qvel[bda + j];
  };
  /* main.xml: the two chains with the components across lanes (r_chain_cols), the several-dof bodies
     (children of the world without children of their own, checked by the generator) on their lanes
     first.  Same expressions, same operands: bit-identical. */
  constexpr bool COLS = KS::STATIC_TREE && UR3E_MAIN_BODY_COLS;
  if constexpr (COLS) {
    if (depth == 1 && bdn > 1) {
      double cv[6];
      for (int k = 0; k < 6; k++) cv[k] = s.cvel[0][k];
      general(cv);
      for (int k = 0; k < 6; k++) s.cvel[lane][k] = cv[k];
    }
    if (depth > 0 && one)
      for (int k = 0; k < 6; k++) s.cvel[lane][k] = cqv[k]; /* staged increment */
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    r_chain_cols<false>(s.cvel);
    if (depth > 0 && one)
      for (int k = 0; k < 6; k++) cvp[k] = s.cvel[pid][k];
  } else {
    /* Split like r_kinematics: the velocity chain cvel = parent cvel + cdof * qvel runs level by level,
       then cdof_dot and the acceleration term of every single-dof body are formed at once, then the
       chain cacc = parent cacc + term.  Same expressions, same operands: bit-identical. */
    for (int lvl = 1; lvl <= nlevel; lvl++) {
      if (depth == lvl) {
        double cv[6];
        for (int k = 0; k < 6; k++) cv[k] = s.cvel[pid][k];
        if (one) {
          for (int r = 0; r < 6; r++) { cvp[r] = cv[r]; cv[r] += cqv[r]; }
        } else {
          general(cv);
        }
        for (int k = 0; k < 6; k++) s.cvel[lane][k] = cv[k];
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
    }
  }
  WT(31);
  if (depth > 0 && one) {
    double cdd[6];
    k_cross_motion(cdd, cvp, cd);
    for (int r = 0; r < 6; r++) cdof_dot[bda][r] = cdd[r];
    for (int r = 0; r < 6; r++) tmp[r] += cdd[r] * qv;
  }
  if constexpr (COLS) {
    if (depth > 0)
      for (int k = 0; k < 6; k++) cacc[lane][k] = tmp[k]; /* staged term (the world's row is set) */
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    r_chain_cols<true>(cacc);
  } else {
    for (int lvl = 1; lvl <= nlevel; lvl++) {
      if (depth == lvl) {
        for (int k = 0; k < 6; k++) cacc[lane][k] = cacc[pid][k] + tmp[k];
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
    }
  }
}

/* body forces of w_rne_passive: cfrc per body, subtree sums in the oracle's order
   (i = nb-1 .. 1, parent += child) as a readlane chain, written to LDS for qfrc_bias */
template <class KS>
WD void r_cfrc(KModel m, KS& s) {
  const int lane = w_lane();
  const int nb = m->nbody;
  auto cacc = w_cacc(s);
  auto cfrc = w_cfrc(s);
  int par[K_NB];
#pragma unroll
  for (int i = 0; i < K_NB; i++) par[i] = m->body_parentid[i];
  double f[6] = {0, 0, 0, 0, 0, 0};
  if (lane >= 1 && lane < nb) {
    double ci[10], ca[6], cv[6];
    for (int k = 0; k < 10; k++) ci[k] = s.cinert[lane][k];
    for (int k = 0; k < 6; k++) { ca[k] = cacc[lane][k]; cv[k] = s.cvel[lane][k]; }
    double f1[6], f2[6], f3[6];
    k_mul_inert_vec(f1, ci, ca);
    k_mul_inert_vec(f2, ci, cv);
    k_cross_force(f3, cv, f2);
    for (int r = 0; r < 6; r++) f[r] = f1[r] + f3[r];
  }
  if constexpr (KS::STATIC_TREE) {
    if (lane < nb)
      for (int r = 0; r < 6; r++) cfrc[lane][r] = f[r]; /* lane 0: the world's zeros */
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    r_subtree_sum_cols<6, true>(cfrc, cfrc);
    return;
  }
#pragma unroll
  for (int i = K_NB - 1; i > 0; i--) {
    if (i < nb) {
      const int p = par[i];
      if (p > 0) {
        double v[6];
#pragma unroll
        for (int r = 0; r < 6; r++) v[r] = rl(f[r], i);
        if (lane == p) {
#pragma unroll
          for (int r = 0; r < 6; r++) f[r] += v[r];
        }
      }
    }
  }
  if (lane < nb) {
    for (int r = 0; r < 6; r++) cfrc[lane][r] = lane == 0 ? 0.0 : f[r];
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

/* ================================================================== */
/* constraint rows for the compact tier: layout and Jacobian            */
/* ================================================================== */
/* Row-group layout in the oracle's order (equality, frictionloss: host-precomputed in KPlan;
   joint limits in (joint, side) order; condim-3 contacts in contact order) by ballot prefix
   sums instead of a serial lane-0 walk.  Any layout that would not fit the compact capacity
   bails (ovf): the full-capacity tier then reproduces the oracle's truncation rule. */
/* the row groups' constants from the host-resolved plan rows (1, default) or through the model's index
   chains (0: A/B) */
#ifndef W_FLAT_GROUPS
#define W_FLAT_GROUPS 1
#endif
template <class KS>
WD void r_mc_layout(KModel m, const KPlan* __restrict__ pl, KS& s) {
  const int lane = w_lane();
  const int nj = m->njnt, ncon = s.ncon;
  int lo = 0, hi = 0;
#if W_FLAT_GROUPS
  /* the joint's limit row of the plan (limited hinge / slide flag, qpos address, margin, range): one load
     level, issued before the test */
  if (lane < nj) {
    const int r = W_CS_JNT + lane;
    const int lim = pl->cs_i[r][1], qa = pl->cs_i[r][2];
    const double mg = pl->cs_d[r][8], rlo = pl->cs_d[r][9], rhi = pl->cs_d[r][10];
    if (lim) {
      const double q = s.qpos[qa];
      const double dlo = -1.0 * (rlo - q);
      const double dhi = 1.0 * (rhi - q);
      lo = dlo < mg;
      hi = dhi < mg;
    }
  }
#else
  if (lane < nj && m->jnt_limited[lane] &&
      (m->jnt_type[lane] == UR3E_JNT_HINGE || m->jnt_type[lane] == UR3E_JNT_SLIDE)) {
    const double q = s.qpos[m->jnt_qposadr[lane]];
    const double mg = m->jnt_margin[lane];
    const double dlo = -1.0 * (m->jnt_range[lane][0] - q);
    const double dhi = 1.0 * (m->jnt_range[lane][1] - q);
    lo = dlo < mg;
    hi = dhi < mg;
  }
#endif
  int c3 = 0;
  if (lane < ncon) c3 = m->cpair_condim[s.con_cpair[lane]] == 3;
  const unsigned long long mlo = __ballot(lo), mhi = __ballot(hi), mc = __ballot(c3);
  const unsigned long long below = lane ? (~0ull >> (64 - lane)) : 0ull;
  const int nfix = pl->nfixgrp, nfixrow = pl->nfixrow;
  const int nlim = __popcll(mlo) + __popcll(mhi);
  const int ncg = __popcll(mc);
  const int nrow = nfixrow + nlim + 3 * ncg;
  const int ngrp = nfix + nlim + ncg;
  /* rows beyond the tier's capacity, or more groups than lanes (lane = group below) or than the layout
     holds (KSX::MAXGRP), bail */
  static_assert(KS::BAIL, "the overlaid layouts hand on what they cannot hold");
  constexpr int GMAX = KS::MAXGRP < 64 ? KS::MAXGRP : 64;
  if (nrow > KS::MAXEFC || ngrp > GMAX) {
    if (lane == 0) s.ovf = 1;
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    return;
  }
  /* group g's rows get type/id/group (+ frictionloss, contact back-pointer) */
  auto put = [&](int g, int type, int id, int r) {
    s.grp_type[g] = type; s.grp_id[g] = id; s.grp_row[g] = r;
    const int n = (type == G_CONNECT || type == G_CONTACT) ? 3 : 1;
    const int ct = type == G_CONNECT || type == G_JOINTEQ ? CN_EQUALITY
                 : type == G_FLOSS ? CN_FRICTION_DOF : type == G_LIMIT ? CN_LIMIT_JOINT : CN_CONTACT_ELLIPTIC;
    const int cid = type == G_LIMIT ? (id >> 1) : id;
    for (int k = 0; k < n; k++) {
      s.efc_type[r + k] = ct; s.efc_id[r + k] = cid; s.efc_grp[r + k] = g;
    }
    if (type == G_CONTACT) s.con_efc[id] = r;
  };
  if (lane < nfix) put(lane, pl->fix_type[lane], pl->fix_id[lane], pl->fix_row[lane]);
  const int loff = __popcll(mlo & below) + __popcll(mhi & below);
  if (lo) put(nfix + loff, G_LIMIT, 2 * lane, nfixrow + loff);
  if (hi) put(nfix + loff + lo, G_LIMIT, 2 * lane + 1, nfixrow + loff + lo);
  if (c3) {
    const int k = __popcll(mc & below);
    put(nfix + nlim + k, G_CONTACT, lane, nfixrow + nlim + 3 * k);
  }
  if (lane == 0) { s.ngrp = ngrp; s.nefc = nrow; }
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

/* Jacobian rows and per-row impedance for the compact tier.
   1. lane = group: the group's geometry (offsets to subtree coms, contact frame, dof masks) and
      its rows' impedance inputs (pos, margin, diag, solref/solimp) into registers;
   2. lane = dof: walk the groups in order, each group's data broadcast by readlane, one code
      path per group type (uniform) -> J columns;
   3. lane = row: fetch its group's inputs by lane shuffle, then one common impedance path.
   Same expressions as w_make_constraint's phases A and B. */
template <class KS>
WD void r_mc_rows(KModel m, const KPlan* __restrict__ pl, KS& s) {
  const int lane = w_lane();
  const int nv = NVOF(KS, m);
  const int ngrp = s.ngrp, nefc = s.nefc;
  /* ---- 1. per-group data (lane = group) ---- */
  int gtype = -1, grow = 0, msk1 = 0, msk2 = 0, dof1 = -1, dof2 = -1, fric = 0;
  double o1[3] = {0, 0, 0}, o2[3] = {0, 0, 0}, fr[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  double gpos[3] = {0, 0, 0}, gmargin = 0, gdiag = 0, dpoly = 0, side = 0;
  double sref[2] = {0, 0}, simp[5] = {0, 0, 0, 0, 0};
#if W_FLAT_GROUPS
  if (lane < ngrp) {
    gtype = s.grp_type[lane];
    const int id = s.grp_id[lane];
    grow = s.grp_row[lane];
    /* the group's constants from its plan row (KPlan.cs_*), all loads one level deep and issued before
       the per-kind branches, which then read only LDS; same values as the index chains below */
    const int src = gtype <= G_JOINTEQ ? id
                    : gtype == G_FLOSS ? W_CS_DOF + id
                    : gtype == G_LIMIT ? W_CS_JNT + (id >> 1)
                                       : W_CS_PAIR + s.con_cpair[id];
    int ci[4];
    double cd[11];
#pragma unroll
    for (int k = 0; k < 4; k++) ci[k] = pl->cs_i[src][k];
#pragma unroll
    for (int k = 0; k < 11; k++) cd[k] = pl->cs_d[src][k];
    for (int k = 0; k < 2; k++) sref[k] = cd[k];
    for (int k = 0; k < 5; k++) simp[k] = cd[2 + k];
    gdiag = cd[7];
    if (gtype == G_CONNECT) {
      const int e = id;
      double p1[3], p2[3];
      for (int k = 0; k < 3; k++) { p1[k] = s.eq_p[e][k]; p2[k] = s.eq_p[e][3 + k]; }
      const int r1 = ci[0], r2 = ci[1];
      for (int k = 0; k < 3; k++) {
        o1[k] = p1[k] - s.subtree_com[r1][k];
        o2[k] = p2[k] - s.subtree_com[r2][k];
        gpos[k] = p1[k] - p2[k];
      }
      msk1 = ci[2]; msk2 = ci[3];
    } else if (gtype == G_JOINTEQ) {
      const double* c = m->eq_data[id];
      dof1 = ci[0];
      const double q1 = s.qpos[ci[2]] - cd[9];
      if (ci[1] >= 0) {
        dof2 = ci[1];
        const double q2 = s.qpos[ci[3]] - cd[10];
        dpoly = c[1] + q2 * (2 * c[2] + q2 * (3 * c[3] + q2 * 4 * c[4]));
        gpos[0] = q1 - (c[0] + q2 * (c[1] + q2 * (c[2] + q2 * (c[3] + q2 * c[4]))));
      } else {
        gpos[0] = q1 - c[0];
      }
    } else if (gtype == G_FLOSS) {
      dof1 = id;
      fric = 1;
    } else if (gtype == G_LIMIT) {
      const int sd = (id & 1) ? 1 : -1;
      side = (double)sd;
      dof1 = ci[0];
      const double q = s.qpos[ci[2]];
      gpos[0] = sd * ((sd > 0 ? cd[10] : cd[9]) - q);
      gmargin = cd[8];
    } else {
      const int c = id;
      const int r1 = ci[0], r2 = ci[1];
      for (int k = 0; k < 3; k++) {
        const double pk = s.con_pos[c][k];
        o1[k] = pk - s.subtree_com[r1][k];
        o2[k] = pk - s.subtree_com[r2][k];
      }
      for (int k = 0; k < 3; k++) fr[k] = s.con_n[c][k];
      k_frame_rest(fr); /* k_make_frame's rows 1-2 from the stored unit normal */
      msk1 = ci[2]; msk2 = ci[3];
      const double d = s.con_dist[c];
      gpos[0] = d; gpos[1] = d; gpos[2] = d;
      gmargin = cd[8];
      fric = 2; /* rows k > 0 */
    }
  }
#else
  if (lane < ngrp) {
    gtype = s.grp_type[lane];
    const int id = s.grp_id[lane];
    grow = s.grp_row[lane];
    if (gtype == G_CONNECT) {
      const int e = id;
      const int b1 = m->eq_obj1[e], b2 = m->eq_obj2[e];
      /* anchors precomputed in w_com_pos (xmat is dead by now) */
      double p1[3], p2[3];
      for (int k = 0; k < 3; k++) { p1[k] = s.eq_p[e][k]; p2[k] = s.eq_p[e][3 + k]; }
      const int r1 = m->body_rootid[b1], r2 = m->body_rootid[b2];
      for (int k = 0; k < 3; k++) {
        o1[k] = p1[k] - s.subtree_com[r1][k];
        o2[k] = p2[k] - s.subtree_com[r2][k];
        gpos[k] = p1[k] - p2[k];
      }
      msk1 = pl->body_dof_mask[b1]; msk2 = pl->body_dof_mask[b2];
      gdiag = m->body_invweight0[b1][0] + m->body_invweight0[b2][0];
      for (int k = 0; k < 2; k++) sref[k] = m->eq_solref[e][k];
      for (int k = 0; k < 5; k++) simp[k] = m->eq_solimp[e][k];
    } else if (gtype == G_JOINTEQ) {
      const int e = id;
      const int j1 = m->eq_obj1[e], j2 = m->eq_obj2[e];
      const double* c = m->eq_data[e];
      dof1 = m->jnt_dofadr[j1];
      const int a1 = m->jnt_qposadr[j1];
      const double q1 = s.qpos[a1] - m->qpos0[a1];
      gdiag = m->dof_invweight0[dof1];
      if (j2 >= 0) {
        dof2 = m->jnt_dofadr[j2];
        const int a2 = m->jnt_qposadr[j2];
        const double q2 = s.qpos[a2] - m->qpos0[a2];
        dpoly = c[1] + q2 * (2 * c[2] + q2 * (3 * c[3] + q2 * 4 * c[4]));
        gpos[0] = q1 - (c[0] + q2 * (c[1] + q2 * (c[2] + q2 * (c[3] + q2 * c[4]))));
        gdiag += m->dof_invweight0[dof2];
      } else {
        gpos[0] = q1 - c[0];
      }
      for (int k = 0; k < 2; k++) sref[k] = m->eq_solref[e][k];
      for (int k = 0; k < 5; k++) simp[k] = m->eq_solimp[e][k];
    } else if (gtype == G_FLOSS) {
      dof1 = id;
      gdiag = m->dof_invweight0[id];
      fric = 1;
      for (int k = 0; k < 2; k++) sref[k] = m->dof_solref[id][k];
      for (int k = 0; k < 5; k++) simp[k] = m->dof_solimp[id][k];
    } else if (gtype == G_LIMIT) {
      const int j = id >> 1;
      const int sd = (id & 1) ? 1 : -1;
      side = (double)sd;
      dof1 = m->jnt_dofadr[j];
      const double q = s.qpos[m->jnt_qposadr[j]];
      gpos[0] = sd * (m->jnt_range[j][(sd + 1) / 2] - q);
      gmargin = m->jnt_margin[j];
      gdiag = m->dof_invweight0[dof1];
      for (int k = 0; k < 2; k++) sref[k] = m->jnt_solref[j][k];
      for (int k = 0; k < 5; k++) simp[k] = m->jnt_solimp[j][k];
    } else {
      const int c = id;
      const int p = s.con_cpair[c];
      const int b1 = m->geom_bodyid[s.con_geom1[c]], b2 = m->geom_bodyid[s.con_geom2[c]];
      const int r1 = m->body_rootid[b1], r2 = m->body_rootid[b2];
      for (int k = 0; k < 3; k++) {
        const double pk = s.con_pos[c][k];
        o1[k] = pk - s.subtree_com[r1][k];
        o2[k] = pk - s.subtree_com[r2][k];
      }
      for (int k = 0; k < 3; k++) fr[k] = s.con_n[c][k];
      k_frame_rest(fr); /* k_make_frame's rows 1-2 from the stored unit normal */
      msk1 = pl->body_dof_mask[b1]; msk2 = pl->body_dof_mask[b2];
      const double d = s.con_dist[c];
      gpos[0] = d; gpos[1] = d; gpos[2] = d;
      gmargin = m->cpair_margin[p] - m->cpair_gap[p];
      gdiag = m->body_invweight0[b1][0] + m->body_invweight0[b2][0];
      fric = 2; /* rows k > 0 */
      for (int k = 0; k < 2; k++) sref[k] = m->cpair_solref[p][k];
      for (int k = 0; k < 5; k++) simp[k] = m->cpair_solimp[p][k];
    }
  }
#endif
  WT(37);
  /* ---- 2. Jacobian: GS groups side by side per pass (lanes [K_NV t, K_NV t + K_NV) take group
     g0 + t, lane = dof within), the group's data by lane shuffle from its group lane, gathered
     with the whole wave active (no permute under divergent control flow) ---- */
  {
    constexpr int GS = 64 / K_NV;
    const int slot = lane / K_NV;
    const int v = lane - slot * K_NV;
    const int vv = v < nv ? v : 0;
    double cd[6];
    for (int r = 0; r < 6; r++) cd[r] = s.cdof[vv][r];
    const unsigned int vbit = 1u << vv;
#if W_MC_TRIVIAL
    /* the unit-vector rows (joint equality, frictionloss, limit: one row each) one group at a time, with
       the group's scalars by readlane and every dof lane writing its entry; the shuffle passes below then
       take only the connect and contact groups, GS at a time in group order */
    const unsigned long long heavy = __ballot(lane < ngrp && (gtype == G_CONNECT || gtype >= G_CONTACT));
    {
      unsigned long long triv = __ballot(lane < ngrp) & ~heavy;
      while (triv) {
        const int g = (int)__builtin_ctzll(triv);
        triv &= triv - 1;
        const int type = rli(gtype, g), r = rli(grow, g), d1 = rli(dof1, g), d2 = rli(dof2, g);
        const double dp = rl(dpoly, g), sd = rl(side, g);
        if (lane < nv) {
          double val;
          if (type == G_JOINTEQ) {
            val = 0;
            if (lane == d1) val = 1;
            if (d2 >= 0 && lane == d2) val = -dp;
          } else if (type == G_FLOSS) {
            val = lane == d1 ? 1.0 : 0.0;
          } else {
            val = lane == d1 ? -sd : 0.0;
          }
          s.efc_J[r][lane] = val;
        }
      }
    }
    const int nheavy = __popcll(heavy);
    unsigned long long hrest = heavy;
    for (int g0 = 0; g0 < nheavy; g0 += GS) {
      /* the groups of heavy ranks g0 .. g0 + GS - 1 (uniform), slot t takes the t-th */
      int gpick = 0;
#pragma unroll
      for (int t = 0; t < GS; t++) {
        const int gt = hrest ? (int)__builtin_ctzll(hrest) : 0;
        hrest &= hrest - 1;
        gpick = slot == t ? gt : gpick;
      }
      const bool on = slot < GS && g0 + slot < nheavy && v < nv;
      const int gs = on ? gpick : 0;
#else
    for (int g0 = 0; g0 < ngrp; g0 += GS) {
      const int g = g0 + slot;
      const bool on = slot < GS && g < ngrp && v < nv;
      const int gs = on ? g : 0;
#endif
      const int type = shfi(gtype, gs), r = shfi(grow, gs);
      const unsigned int m1 = (unsigned int)shfi(msk1, gs), m2 = (unsigned int)shfi(msk2, gs);
      const int d1 = shfi(dof1, gs), d2 = shfi(dof2, gs);
      double a1[3], a2[3], f[9];
      for (int k = 0; k < 3; k++) { a1[k] = shf(o1[k], gs); a2[k] = shf(o2[k], gs); }
      for (int k = 0; k < 9; k++) f[k] = shf(fr[k], gs);
      const double dp = shf(dpoly, gs), sd = shf(side, gs);
      if (on) {
        if (type == G_CONNECT || type >= G_CONTACT) {
          double j1[3], j2[3];
          if (m1 & vbit) {
            double cr[3];
            k_cross3(cr, cd, a1);
            j1[0] = cd[3] + cr[0]; j1[1] = cd[4] + cr[1]; j1[2] = cd[5] + cr[2];
          } else {
            j1[0] = 0; j1[1] = 0; j1[2] = 0;
          }
          if (m2 & vbit) {
            double cr[3];
            k_cross3(cr, cd, a2);
            j2[0] = cd[3] + cr[0]; j2[1] = cd[4] + cr[1]; j2[2] = cd[5] + cr[2];
          } else {
            j2[0] = 0; j2[1] = 0; j2[2] = 0;
          }
          if (type == G_CONNECT) {
            for (int k = 0; k < 3; k++) s.efc_J[r + k][v] = j1[k] - j2[k];
          } else {
            const double dj0 = j2[0] - j1[0], dj1 = j2[1] - j1[1], dj2 = j2[2] - j1[2];
            for (int k = 0; k < 3; k++) s.efc_J[r + k][v] = f[3 * k] * dj0 + f[3 * k + 1] * dj1 + f[3 * k + 2] * dj2;
          }
        } else if (type == G_JOINTEQ) {
          double val = 0;
          if (v == d1) val = 1;
          if (d2 >= 0 && v == d2) val = -dp;
          s.efc_J[r][v] = val;
        } else if (type == G_FLOSS) {
          s.efc_J[r][v] = v == d1 ? 1.0 : 0.0;
        } else {
          s.efc_J[r][v] = v == d1 ? -sd : 0.0;
        }
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  WT(38);
  /* ---- 3. impedance, lane = row (w_row_impedance); row lane + 64 h for each row slot ---- */
  constexpr int SPLIT = KS::STATIC_TREE ? UR3E_MAIN_SPLIT : 0;
  int couples = 0; /* a row of this lane has nonzeros in both dof trees */
#pragma unroll
  for (int h = 0; h < KS::RPL; h++) {
    int t2only = 0; /* the row has no nonzero in the first dof tree [0, SPLIT) */
    const int r = lane + 64 * h;
    const int g = r < nefc ? s.efc_grp[r] : 0;
    const int k = r < nefc ? r - s.grp_row[g] : 0;
    const double p0 = shf(gpos[0], g), p1 = shf(gpos[1], g), p2 = shf(gpos[2], g);
    const double pos = k == 0 ? p0 : (k == 1 ? p1 : p2);
    const double margin = shf(gmargin, g), diag = shf(gdiag, g);
    const int fr_ = shfi(fric, g);
    const int friction_row = fr_ == 1 || (fr_ == 2 && k > 0);
    double sr[2], si[5];
    for (int q = 0; q < 2; q++) sr[q] = shf(sref[q], g);
    for (int q = 0; q < 5; q++) si[q] = shf(simp[q], g);
    if (r < nefc) {
      double jr[K_NV], qv[K_NV];
#pragma unroll
      for (int q = 0; q < K_NV; q++) { jr[q] = s.efc_J[r][q]; qv[q] = s.qvel[q]; }
      double vel = 0;
#pragma unroll
      for (int q = 0; q < K_NV; q++)
        if (q < nv) vel += jr[q] * qv[q];
      if constexpr (SPLIT > 0) {
        bool a = false, b = false;
#pragma unroll
        for (int q = 0; q < K_NV; q++)
          if (q < nv) {
            if (q < SPLIT) a = a || jr[q] != 0;
            else b = b || jr[q] != 0;
          }
        couples |= a && b;
        t2only = !a;
      }
      double imp = k_get_impedance(si, pos, margin);
      double dmax = si[1];
      if (dmax < K_MINIMP) dmax = K_MINIMP;
      if (dmax > K_MAXIMP) dmax = K_MAXIMP;
      double K, B;
      if (sr[0] > 0) {
        double tc = sr[0];
        if (tc < 2 * m->timestep) tc = 2 * m->timestep;
        double dr = sr[1];
        K = 1.0 / (dmax * dmax * tc * tc * dr * dr);
        B = 2.0 / (dmax * tc);
      } else {
        K = -sr[0] / (dmax * dmax);
        B = -sr[1] / dmax;
      }
      if (friction_row)
        s.efc_aref[r] = -B * vel;
      else
        s.efc_aref[r] = -B * vel - K * imp * (pos - margin);
      double R = (1 - imp) * diag / imp;
      s.efc_R[r] = R < K_MINVAL ? K_MINVAL : R;
    }
#if W_T2_SKIP
    if constexpr (SPLIT > 0) {
      const unsigned long long t2m = __ballot(t2only);
      if (lane == 0) s.t2rows[h] = t2m;
    }
#endif
  }
  if constexpr (SPLIT > 0) {
    const bool any = __ballot(couples) != 0;
    if (lane == 0) s.bdiag = !any;
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

#endif /* UR3E_WAVE_R_H */
