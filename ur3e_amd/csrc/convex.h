/*
 * convex.h — narrowphase for convex mesh geoms (type mesh, MuJoCo numbering 7): plane–convex,
 * and convex–convex (box–mesh, mesh–mesh) by GJK + EPA.  One source for the GPU tiers and the CPU
 * oracle (plain C99 with UR3E_HD qualifiers, like detmath.h), compiled with -ffp-contract=off on both
 * sides, so the contacts are bit-identical.
 *
 * Semantics restated from MuJoCo 3.3.3's documented convex collision (Computation chapter, "Collision
 * detection"): a mesh collides through its convex hull; plane–convex keeps the hull vertices within
 * the margin of the plane (at most UR3E_CVX_PLANE_MAX of them, deepest first, then in vertex order),
 * each contact halfway between the vertex and its projection, normal = plane normal; a pair of convex
 * shapes gives ONE contact (MuJoCo's default without the multiccd flag): GJK decides separation and,
 * for separated shapes within the margin, the closest points; EPA on the Minkowski difference gives
 * the penetration depth and direction of overlapping shapes.  The contact normal points from geom1 to
 * geom2, dist < 0 is penetration, pos is the midpoint of the two witness points.  MuJoCo's own
 * GJK/EPA (engine_collision_gjk.c) and plane–convex routine are not in this image, so parity with
 * MuJoCo itself is unpinned; tests/test_mesh.py pins these routines to closed forms (box as a mesh
 * against the box primitives' contacts and penetration depths).
 */
#ifndef UR3E_CONVEX_H
#define UR3E_CONVEX_H

#if defined(__HIPCC__)
#define UR3E_HD __host__ __device__ static inline
#else
#ifndef UR3E_HD
#define UR3E_HD static inline
#endif
#endif

#include <math.h>

#define UR3E_CVX_PLANE_MAX 4   /* plane–convex contacts */
#define UR3E_GJK_ITERS 64
#define UR3E_EPA_ITERS 48
#define UR3E_EPA_MAXV (4 + UR3E_EPA_ITERS)
#define UR3E_EPA_MAXF (4 + 2 * UR3E_EPA_ITERS + 8)
#define UR3E_GJK_TOL 1e-12
#define UR3E_EPA_TOL 1e-10

/* a convex shape in world coordinates: box (v == 0: half sizes) or hull vertices in the geom frame */
typedef struct {
  const double* v; /* nv * 3 local vertices (mesh) or 0 (box) */
  int nv;
  double size[3];
  double pos[3];
  double mat[9];   /* row-major geom_xmat */
} ur3e_cvx;

UR3E_HD double ur3e_cvx_dot(const double a[3], const double b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
UR3E_HD void ur3e_cvx_sub(double r[3], const double a[3], const double b[3]) {
  r[0] = a[0] - b[0]; r[1] = a[1] - b[1]; r[2] = a[2] - b[2];
}
UR3E_HD void ur3e_cvx_cross(double r[3], const double a[3], const double b[3]) {
  r[0] = a[1] * b[2] - a[2] * b[1];
  r[1] = a[2] * b[0] - a[0] * b[2];
  r[2] = a[0] * b[1] - a[1] * b[0];
}

/* support point of shape c in world direction d (the first vertex reaching the maximum) */
UR3E_HD void ur3e_cvx_support(const ur3e_cvx* c, const double d[3], double out[3]) {
  const double* R = c->mat;
  const double ld0 = R[0] * d[0] + R[3] * d[1] + R[6] * d[2];
  const double ld1 = R[1] * d[0] + R[4] * d[1] + R[7] * d[2];
  const double ld2 = R[2] * d[0] + R[5] * d[1] + R[8] * d[2];
  double l0, l1, l2;
  if (c->v) {
    int best = 0;
    double bd = c->v[0] * ld0 + c->v[1] * ld1 + c->v[2] * ld2;
    for (int k = 1; k < c->nv; k++) {
      const double dd = c->v[3 * k] * ld0 + c->v[3 * k + 1] * ld1 + c->v[3 * k + 2] * ld2;
      if (dd > bd) { bd = dd; best = k; }
    }
    l0 = c->v[3 * best]; l1 = c->v[3 * best + 1]; l2 = c->v[3 * best + 2];
  } else {
    l0 = ld0 >= 0 ? c->size[0] : -c->size[0];
    l1 = ld1 >= 0 ? c->size[1] : -c->size[1];
    l2 = ld2 >= 0 ? c->size[2] : -c->size[2];
  }
  out[0] = c->pos[0] + R[0] * l0 + R[1] * l1 + R[2] * l2;
  out[1] = c->pos[1] + R[3] * l0 + R[4] * l1 + R[5] * l2;
  out[2] = c->pos[2] + R[6] * l0 + R[7] * l1 + R[8] * l2;
}

/* ---- plane (geom1: normal = z axis of its frame) vs convex hull (geom2) --------------------- */
UR3E_HD int ur3e_plane_convex(const double pp[3], const double pm[9], const ur3e_cvx* c, double margin,
                              double pos[][3], double nrm[][3], double* dist) {
  const double n[3] = {pm[2], pm[5], pm[8]};
  double dif[3];
  ur3e_cvx_sub(dif, c->pos, pp);
  const double d0 = ur3e_cvx_dot(n, dif);
  int sel[UR3E_CVX_PLANE_MAX];
  double sd[UR3E_CVX_PLANE_MAX];
  int ns = 0;
  const double* R = c->mat;
  for (int k = 0; k < c->nv; k++) {
    const double* v = c->v + 3 * k;
    double w[3];
    w[0] = R[0] * v[0] + R[1] * v[1] + R[2] * v[2];
    w[1] = R[3] * v[0] + R[4] * v[1] + R[5] * v[2];
    w[2] = R[6] * v[0] + R[7] * v[1] + R[8] * v[2];
    const double dd = d0 + ur3e_cvx_dot(n, w);
    if (dd > margin) continue;
    if (ns < UR3E_CVX_PLANE_MAX) {
      sel[ns] = k; sd[ns] = dd; ns++;
    } else { /* replace the shallowest kept vertex if this one is deeper */
      int worst = 0;
      for (int j = 1; j < ns; j++)
        if (sd[j] > sd[worst]) worst = j;
      if (dd < sd[worst]) { sel[worst] = k; sd[worst] = dd; }
    }
  }
  /* output deepest first (ties: lower vertex index first) */
  for (int i = 0; i < ns; i++) {
    int b = i;
    for (int j = i + 1; j < ns; j++)
      if (sd[j] < sd[b] || (sd[j] == sd[b] && sel[j] < sel[b])) b = j;
    const int tk = sel[i]; sel[i] = sel[b]; sel[b] = tk;
    const double td = sd[i]; sd[i] = sd[b]; sd[b] = td;
    const double* v = c->v + 3 * sel[i];
    double w[3];
    w[0] = R[0] * v[0] + R[1] * v[1] + R[2] * v[2];
    w[1] = R[3] * v[0] + R[4] * v[1] + R[5] * v[2];
    w[2] = R[6] * v[0] + R[7] * v[1] + R[8] * v[2];
    const double h = sd[i] * 0.5;
    pos[i][0] = c->pos[0] + w[0] - n[0] * h;
    pos[i][1] = c->pos[1] + w[1] - n[1] * h;
    pos[i][2] = c->pos[2] + w[2] - n[2] * h;
    nrm[i][0] = n[0]; nrm[i][1] = n[1]; nrm[i][2] = n[2];
    dist[i] = sd[i];
  }
  return ns;
}

/* ---- GJK on the Minkowski difference A - B ------------------------------------------------- */
typedef struct {
  double w[4][3];  /* a - b */
  double a[4][3];  /* support points of A */
  double b[4][3];  /* support points of B */
  int n;
} ur3e_simplex;

UR3E_HD void ur3e_simplex_keep(ur3e_simplex* s, int i0, int i1, int i2, int n) {
  const int idx[3] = {i0, i1, i2};
  double w[3][3], a[3][3], b[3][3];
  for (int k = 0; k < n; k++)
    for (int c = 0; c < 3; c++) {
      w[k][c] = s->w[idx[k]][c]; a[k][c] = s->a[idx[k]][c]; b[k][c] = s->b[idx[k]][c];
    }
  for (int k = 0; k < n; k++)
    for (int c = 0; c < 3; c++) {
      s->w[k][c] = w[k][c]; s->a[k][c] = a[k][c]; s->b[k][c] = b[k][c];
    }
  s->n = n;
}

/* keep simplex vertex i alone */
UR3E_HD void ur3e_sx_vertex(ur3e_simplex* s, int i, double v[3], double lam[4]) {
  ur3e_simplex_keep(s, i, 0, 0, 1);
  v[0] = s->w[0][0]; v[1] = s->w[0][1]; v[2] = s->w[0][2];
  lam[0] = 1;
}
/* keep the edge (i, j) with the point w_i + u (w_j - w_i) */
UR3E_HD void ur3e_sx_edge(ur3e_simplex* s, int i, int j, double u, double v[3], double lam[4]) {
  ur3e_simplex_keep(s, i, j, 0, 2);
  lam[0] = 1 - u; lam[1] = u;
  for (int c = 0; c < 3; c++) v[c] = s->w[0][c] + u * (s->w[1][c] - s->w[0][c]);
}

/* closest point to the origin of the triangle (w0, w1, w2), reducing s to its supporting feature
   (Ericson, Real-Time Collision Detection 5.1.5, ClosestPtPointTriangle with p = origin) */
UR3E_HD void ur3e_sx_triangle(ur3e_simplex* s, double v[3], double lam[4]) {
  const double *A = s->w[0], *B = s->w[1], *C = s->w[2];
  double ab[3], ac[3];
  ur3e_cvx_sub(ab, B, A); ur3e_cvx_sub(ac, C, A);
  const double ap[3] = {-A[0], -A[1], -A[2]};
  const double d1 = ur3e_cvx_dot(ab, ap), d2 = ur3e_cvx_dot(ac, ap);
  if (d1 <= 0 && d2 <= 0) { ur3e_sx_vertex(s, 0, v, lam); return; }
  const double bp[3] = {-B[0], -B[1], -B[2]};
  const double d3 = ur3e_cvx_dot(ab, bp), d4 = ur3e_cvx_dot(ac, bp);
  if (d3 >= 0 && d4 <= d3) { ur3e_sx_vertex(s, 1, v, lam); return; }
  const double vc = d1 * d4 - d3 * d2;
  if (vc <= 0 && d1 >= 0 && d3 <= 0) { ur3e_sx_edge(s, 0, 1, d1 / (d1 - d3), v, lam); return; }
  const double cp[3] = {-C[0], -C[1], -C[2]};
  const double d5 = ur3e_cvx_dot(ab, cp), d6 = ur3e_cvx_dot(ac, cp);
  if (d6 >= 0 && d5 <= d6) { ur3e_sx_vertex(s, 2, v, lam); return; }
  const double vb = d5 * d2 - d1 * d6;
  if (vb <= 0 && d2 >= 0 && d6 <= 0) { ur3e_sx_edge(s, 0, 2, d2 / (d2 - d6), v, lam); return; }
  const double va = d3 * d6 - d5 * d4;
  if (va <= 0 && (d4 - d3) >= 0 && (d5 - d6) >= 0) {
    ur3e_sx_edge(s, 1, 2, (d4 - d3) / ((d4 - d3) + (d5 - d6)), v, lam);
    return;
  }
  const double den = va + vb + vc;
  if (!(den > 0)) { /* degenerate (flat) triangle: its first edge */
    const double t = d1, dd = ur3e_cvx_dot(ab, ab);
    if (!(t > 0) || !(dd > 0)) { ur3e_sx_vertex(s, 0, v, lam); return; }
    if (t >= dd) { ur3e_sx_vertex(s, 1, v, lam); return; }
    ur3e_sx_edge(s, 0, 1, t / dd, v, lam);
    return;
  }
  const double vv = vb / den, ww = vc / den;
  lam[0] = 1 - vv - ww; lam[1] = vv; lam[2] = ww;
  for (int c = 0; c < 3; c++) v[c] = A[c] + ab[c] * vv + ac[c] * ww;
}

/* closest point of the current simplex to the origin, reducing the simplex to the supporting
   feature; lam[] are its barycentric weights; returns 1 when the origin lies inside the tetrahedron
   (overlap) */
UR3E_HD int ur3e_simplex_closest(ur3e_simplex* s, double v[3], double lam[4]) {
  if (s->n == 1) {
    v[0] = s->w[0][0]; v[1] = s->w[0][1]; v[2] = s->w[0][2];
    lam[0] = 1;
    return 0;
  }
  if (s->n == 2) {
    double ab[3];
    ur3e_cvx_sub(ab, s->w[1], s->w[0]);
    const double ao[3] = {-s->w[0][0], -s->w[0][1], -s->w[0][2]};
    const double t = ur3e_cvx_dot(ao, ab), dd = ur3e_cvx_dot(ab, ab);
    if (!(t > 0) || !(dd > 0)) { ur3e_sx_vertex(s, 0, v, lam); return 0; }
    if (t >= dd) { ur3e_sx_vertex(s, 1, v, lam); return 0; }
    ur3e_sx_edge(s, 0, 1, t / dd, v, lam);
    return 0;
  }
  if (s->n == 3) {
    ur3e_sx_triangle(s, v, lam);
    return 0;
  }
  /* tetrahedron: the origin inside all four faces (oriented away from the opposite vertex) -> overlap;
     else the closest point of the nearest face that has the origin outside */
  {
    const int F[4][4] = {{0, 1, 2, 3}, {0, 3, 1, 2}, {0, 2, 3, 1}, {1, 3, 2, 0}};
    double best = 1e300;
    int bf = -1;
    double bv[3] = {0, 0, 0}, bl[4] = {0, 0, 0, 0};
    ur3e_simplex bs = *s;
    for (int f = 0; f < 4; f++) {
      const double *A = s->w[F[f][0]], *B = s->w[F[f][1]], *C = s->w[F[f][2]], *D = s->w[F[f][3]];
      double ab[3], ac[3], nn[3], ad[3];
      ur3e_cvx_sub(ab, B, A); ur3e_cvx_sub(ac, C, A); ur3e_cvx_cross(nn, ab, ac);
      ur3e_cvx_sub(ad, D, A);
      const double sd = ur3e_cvx_dot(nn, ad);
      const double so = -ur3e_cvx_dot(nn, A);
      /* origin on the other side of the face than D (or the tetrahedron is flat: test every face) */
      if (sd * so < 0 || sd == 0) {
        ur3e_simplex t = *s;
        ur3e_simplex_keep(&t, F[f][0], F[f][1], F[f][2], 3);
        double tv[3], tl[4] = {0, 0, 0, 0};
        ur3e_sx_triangle(&t, tv, tl);
        const double dd = ur3e_cvx_dot(tv, tv);
        if (dd < best) {
          best = dd; bf = f; bs = t;
          bv[0] = tv[0]; bv[1] = tv[1]; bv[2] = tv[2];
          bl[0] = tl[0]; bl[1] = tl[1]; bl[2] = tl[2]; bl[3] = tl[3];
        }
      }
    }
    if (bf < 0) {
      v[0] = 0; v[1] = 0; v[2] = 0;
      return 1;
    }
    *s = bs;
    v[0] = bv[0]; v[1] = bv[1]; v[2] = bv[2];
    lam[0] = bl[0]; lam[1] = bl[1]; lam[2] = bl[2]; lam[3] = bl[3];
    return 0;
  }
}

UR3E_HD void ur3e_mink_support(const ur3e_cvx* A, const ur3e_cvx* B, const double d[3], double a[3], double b[3],
                               double w[3]) {
  const double nd[3] = {-d[0], -d[1], -d[2]};
  ur3e_cvx_support(A, d, a);
  ur3e_cvx_support(B, nd, b);
  ur3e_cvx_sub(w, a, b);
}

/* GJK: returns 1 on overlap (s holds a tetrahedron enclosing the origin, or a lower simplex touching
   it), 0 when separated, with the closest points pa (on A) and pb (on B).
   cut >= 0: returns 2 as soon as a support point proves the shapes farther apart than cut.  The new
   support w = s_{A-B}(-v) bounds A - B by the plane {x : x.v >= w.v}, so dist(A, B) >= w.v / |v|; a caller
   that only needs to know whether the distance exceeds a margin (every caller here: a pair farther apart
   than its margin gives no contact) stops there instead of refining the closest points.  The exit also
   keeps certainly-separated pairs away from the tetrahedron test below, which on a nearly flat simplex
   could report the origin inside for hulls that are apart (round 5: two such pairs in the holding-pose
   test, tests/test_gpu_mesh_main.py, gave EPA "contacts" with positive distance). */
UR3E_HD int ur3e_gjk(const ur3e_cvx* A, const ur3e_cvx* B, ur3e_simplex* s, double pa[3], double pb[3],
                     double cut) {
  double d[3];
  ur3e_cvx_sub(d, B->pos, A->pos); /* initial direction: toward A - B's origin side */
  d[0] = -d[0]; d[1] = -d[1]; d[2] = -d[2];
  if (d[0] == 0 && d[1] == 0 && d[2] == 0) d[0] = 1;
  s->n = 1;
  ur3e_mink_support(A, B, d, s->a[0], s->b[0], s->w[0]);
  double v[3], lam[4];
  v[0] = s->w[0][0]; v[1] = s->w[0][1]; v[2] = s->w[0][2];
  lam[0] = 1; lam[1] = 0; lam[2] = 0; lam[3] = 0;
  for (int it = 0; it < UR3E_GJK_ITERS; it++) {
    const double vv = ur3e_cvx_dot(v, v);
    if (vv <= 1e-30) return 1; /* the origin is on the simplex: touching / overlap */
    const double nd[3] = {-v[0], -v[1], -v[2]};
    double a[3], b[3], w[3];
    ur3e_mink_support(A, B, nd, a, b, w);
    const double vw = ur3e_cvx_dot(v, w);
    if (cut >= 0 && vw > 0 && vw * vw > cut * cut * vv) return 2; /* apart beyond cut */
    /* no progress toward the origin: v is the minimum distance vector */
    if (vv - vw <= UR3E_GJK_TOL * vv) break;
    const int k = s->n;
    for (int c = 0; c < 3; c++) { s->w[k][c] = w[c]; s->a[k][c] = a[c]; s->b[k][c] = b[c]; }
    s->n = k + 1;
    if (ur3e_simplex_closest(s, v, lam)) return 1;
  }
  for (int c = 0; c < 3; c++) {
    double xa = 0, xb = 0;
    for (int k = 0; k < s->n; k++) { xa += lam[k] * s->a[k][c]; xb += lam[k] * s->b[k][c]; }
    pa[c] = xa; pb[c] = xb;
  }
  return 0;
}

/* UR3E_GJK_CUT_SLACK: the separating-axis certificate's slack over the margin, above the rounding of
   w.v (~1e-15 at these scales) */
#define UR3E_GJK_CUT_SLACK 1e-9

/* ---- EPA: penetration of overlapping A, B from a GJK simplex --------------------------------- */
typedef struct {
  double w[UR3E_EPA_MAXV][3], a[UR3E_EPA_MAXV][3], b[UR3E_EPA_MAXV][3];
  int nv;
  int f[UR3E_EPA_MAXF][3];
  double fn[UR3E_EPA_MAXF][3]; /* unit outward normal */
  double fd[UR3E_EPA_MAXF];    /* distance of the face plane from the origin */
  int alive[UR3E_EPA_MAXF];
  int nf;
} ur3e_epa;

/* add face (i, j, k).  orient = 1 (the initial tetrahedron, whose winding is arbitrary): wind it so that
   its normal points away from the origin, which lies inside.  orient = 0 (a horizon face (i, j, new
   vertex), with the edge (i, j) in the winding of the removed face it bordered): the winding is already
   outward, so the normal follows it and the plane offset keeps its sign -- when the origin lies on or
   within rounding of the face plane (touching and shallow contacts), a sign test could flip the normal
   inward and reverse the contact normal. */
UR3E_HD int ur3e_epa_face(ur3e_epa* P, int i, int j, int k, int orient) {
  if (P->nf >= UR3E_EPA_MAXF) return -1;
  double ab[3], ac[3], n[3];
  ur3e_cvx_sub(ab, P->w[j], P->w[i]);
  ur3e_cvx_sub(ac, P->w[k], P->w[i]);
  ur3e_cvx_cross(n, ab, ac);
  const double len = sqrt(ur3e_cvx_dot(n, n));
  if (!(len > 0)) return -1;
  n[0] /= len; n[1] /= len; n[2] /= len;
  double d = ur3e_cvx_dot(n, P->w[i]);
  int f = P->nf++;
  if (orient && d < 0) {
    P->f[f][0] = i; P->f[f][1] = k; P->f[f][2] = j;
    n[0] = -n[0]; n[1] = -n[1]; n[2] = -n[2];
    d = -d;
  } else {
    P->f[f][0] = i; P->f[f][1] = j; P->f[f][2] = k;
  }
  P->fn[f][0] = n[0]; P->fn[f][1] = n[1]; P->fn[f][2] = n[2];
  P->fd[f] = d;
  P->alive[f] = 1;
  return f;
}

UR3E_HD int ur3e_epa_addv(ur3e_epa* P, const double w[3], const double a[3], const double b[3]) {
  if (P->nv >= UR3E_EPA_MAXV) return -1;
  const int k = P->nv++;
  for (int c = 0; c < 3; c++) { P->w[k][c] = w[c]; P->a[k][c] = a[c]; P->b[k][c] = b[c]; }
  return k;
}

/* grow a GJK simplex of 1-3 points to a tetrahedron around the origin (support along fixed axes) */
UR3E_HD int ur3e_epa_seed(const ur3e_cvx* A, const ur3e_cvx* B, ur3e_simplex* s) {
  const double dirs[6][3] = {{1, 0, 0}, {-1, 0, 0}, {0, 1, 0}, {0, -1, 0}, {0, 0, 1}, {0, 0, -1}};
  for (int q = 0; q < 6 && s->n < 4; q++) {
    double a[3], b[3], w[3];
    ur3e_mink_support(A, B, dirs[q], a, b, w);
    int dup = 0;
    for (int k = 0; k < s->n; k++) {
      double e[3];
      ur3e_cvx_sub(e, w, s->w[k]);
      if (ur3e_cvx_dot(e, e) < 1e-24) dup = 1;
    }
    if (s->n == 2 && !dup) { /* reject collinear */
      double e1[3], e2[3], cr[3];
      ur3e_cvx_sub(e1, s->w[1], s->w[0]); ur3e_cvx_sub(e2, w, s->w[0]); ur3e_cvx_cross(cr, e1, e2);
      if (ur3e_cvx_dot(cr, cr) < 1e-24) dup = 1;
    }
    if (s->n == 3 && !dup) { /* reject coplanar */
      double e1[3], e2[3], e3[3], cr[3];
      ur3e_cvx_sub(e1, s->w[1], s->w[0]); ur3e_cvx_sub(e2, s->w[2], s->w[0]); ur3e_cvx_sub(e3, w, s->w[0]);
      ur3e_cvx_cross(cr, e1, e2);
      const double vol = ur3e_cvx_dot(cr, e3);
      if (vol * vol < 1e-36) dup = 1;
    }
    if (dup) continue;
    const int k = s->n++;
    for (int c = 0; c < 3; c++) { s->w[k][c] = w[c]; s->a[k][c] = a[c]; s->b[k][c] = b[c]; }
  }
  return s->n == 4;
}

/* penetration depth and contact: returns 1 with n (unit, from A to B), depth >= 0, pa, pb witnesses */
UR3E_HD int ur3e_epa_run(const ur3e_cvx* A, const ur3e_cvx* B, ur3e_simplex* s, ur3e_epa* P, double n[3],
                         double* depth, double pa[3], double pb[3]) {
  if (s->n < 4 && !ur3e_epa_seed(A, B, s)) return 0;
  P->nv = 0; P->nf = 0;
  for (int k = 0; k < 4; k++) ur3e_epa_addv(P, s->w[k], s->a[k], s->b[k]);
  if (ur3e_epa_face(P, 0, 1, 2, 1) < 0 || ur3e_epa_face(P, 0, 3, 1, 1) < 0 || ur3e_epa_face(P, 0, 2, 3, 1) < 0 ||
      ur3e_epa_face(P, 1, 3, 2, 1) < 0)
    return 0;
  int best = 0;
  for (int it = 0; it < UR3E_EPA_ITERS; it++) {
    best = -1;
    for (int f = 0; f < P->nf; f++)
      if (P->alive[f] && (best < 0 || P->fd[f] < P->fd[best])) best = f;
    if (best < 0) return 0;
    double a[3], b[3], w[3];
    ur3e_mink_support(A, B, P->fn[best], a, b, w);
    const double dw = ur3e_cvx_dot(P->fn[best], w);
    if (dw - P->fd[best] <= UR3E_EPA_TOL) break;
    const int nvx = ur3e_epa_addv(P, w, a, b);
    if (nvx < 0) break;
    /* remove the faces that see w, collect their horizon edges (edges of exactly one removed face) */
    int edges[3 * UR3E_EPA_MAXF][2];
    int ne = 0;
    for (int f = 0; f < P->nf; f++) {
      if (!P->alive[f]) continue;
      double dv[3];
      ur3e_cvx_sub(dv, w, P->w[P->f[f][0]]);
      if (ur3e_cvx_dot(P->fn[f], dv) <= 0) continue;
      P->alive[f] = 0;
      for (int e = 0; e < 3; e++) {
        const int i = P->f[f][e], j = P->f[f][(e + 1) % 3];
        int found = -1;
        for (int q = 0; q < ne; q++)
          if (edges[q][0] == j && edges[q][1] == i) found = q;
        if (found >= 0) { /* shared by two removed faces: not on the horizon */
          edges[found][0] = edges[ne - 1][0]; edges[found][1] = edges[ne - 1][1];
          ne--;
        } else if (ne < 3 * UR3E_EPA_MAXF) {
          edges[ne][0] = i; edges[ne][1] = j; ne++;
        }
      }
    }
    int ok = 1;
    for (int q = 0; q < ne; q++)
      if (ur3e_epa_face(P, edges[q][0], edges[q][1], nvx, 0) < 0) ok = 0;
    if (!ok) break;
  }
  /* contact from the closest face: the origin's projection in barycentric coordinates */
  best = -1;
  for (int f = 0; f < P->nf; f++)
    if (P->alive[f] && (best < 0 || P->fd[f] < P->fd[best])) best = f;
  if (best < 0) return 0;
  const int i0 = P->f[best][0], i1 = P->f[best][1], i2 = P->f[best][2];
  double p[3] = {P->fn[best][0] * P->fd[best], P->fn[best][1] * P->fd[best], P->fn[best][2] * P->fd[best]};
  double v0[3], v1[3], v2[3];
  ur3e_cvx_sub(v0, P->w[i1], P->w[i0]); ur3e_cvx_sub(v1, P->w[i2], P->w[i0]); ur3e_cvx_sub(v2, p, P->w[i0]);
  const double d00 = ur3e_cvx_dot(v0, v0), d01 = ur3e_cvx_dot(v0, v1), d11 = ur3e_cvx_dot(v1, v1);
  const double d20 = ur3e_cvx_dot(v2, v0), d21 = ur3e_cvx_dot(v2, v1);
  const double den = d00 * d11 - d01 * d01;
  double l1 = 0, l2 = 0;
  if (den > 0) { l1 = (d11 * d20 - d01 * d21) / den; l2 = (d00 * d21 - d01 * d20) / den; }
  const double l0 = 1 - l1 - l2;
  for (int c = 0; c < 3; c++) {
    pa[c] = l0 * P->a[i0][c] + l1 * P->a[i1][c] + l2 * P->a[i2][c];
    pb[c] = l0 * P->b[i0][c] + l1 * P->b[i1][c] + l2 * P->b[i2][c];
  }
  /* the origin leaves A - B through this face when B moves by fd * fn: B lies on the +fn side of A,
     so fn is the contact normal from A to B */
  n[0] = P->fn[best][0]; n[1] = P->fn[best][1]; n[2] = P->fn[best][2];
  *depth = P->fd[best];
  return 1;
}

/* one contact between convex shapes A (geom1) and B (geom2) within `margin`; returns 0 or 1 */
UR3E_HD int ur3e_convex_convex(const ur3e_cvx* A, const ur3e_cvx* B, double margin, ur3e_epa* scratch,
                               double pos[3], double nrm[3], double* dist) {
  ur3e_simplex s;
  double pa[3], pb[3];
  const int g = ur3e_gjk(A, B, &s, pa, pb, margin + UR3E_GJK_CUT_SLACK);
  if (g == 2) return 0; /* apart beyond the margin: no contact */
  if (!g) {
    double dv[3];
    ur3e_cvx_sub(dv, pb, pa);
    const double dd = sqrt(ur3e_cvx_dot(dv, dv));
    if (!(dd <= margin) || !(dd > 0)) return 0;
    nrm[0] = dv[0] / dd; nrm[1] = dv[1] / dd; nrm[2] = dv[2] / dd;
    for (int c = 0; c < 3; c++) pos[c] = 0.5 * (pa[c] + pb[c]);
    *dist = dd;
    return 1;
  }
  double n[3], depth;
  if (!ur3e_epa_run(A, B, &s, scratch, n, &depth, pa, pb)) return 0;
  nrm[0] = n[0]; nrm[1] = n[1]; nrm[2] = n[2];
  for (int c = 0; c < 3; c++) pos[c] = 0.5 * (pa[c] + pb[c]);
  *dist = -depth;
  return 1;
}

#endif /* UR3E_CONVEX_H */
