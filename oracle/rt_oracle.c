/* rt_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline "port").
 *
 * Plain-C restatement of plindhorst/Ray-Tracing-Project's CPU ray tracer. Every function cites the
 * reference file:line it restates. Float arithmetic follows Eigen 3.3.7's evaluation order
 * (pinned by tests/golden/eigen_kat.bin). Build WITHOUT FMA contraction (oracle/Makefile:
 * -ffp-contract=off, no -march): the reference is compiled for baseline x86-64 (SSE2, no FMA).
 *
 * Deliberate, result-preserving differences from the reference:
 *   - loop-invariant work is hoisted: getShapeModelMatrix()/inverse() (flyscene.cpp:485-487,446,573)
 *     are computed once, world vertices and normalised face/vertex normals once per mesh; each is
 *     the same float expression evaluated once instead of per call, so bits are unchanged;
 *   - Face objects are not copied per triangle test (flyscene.cpp:385): indices are used;
 *   - every W x H pixel is traced (the reference's `i < h` column bug, flyscene.cpp:306, and its
 *     H%20 / H>=1000 constraints, :269-284, are entry-point bugs, not hot-path semantics);
 *   - the sticky Flyscene material members (flyscene.hpp:179-184, written at flyscene.cpp:356-357,
 *     548-553) are reset to their defaults at the start of every pixel. For scenes where every face
 *     has a material, or none does, this equals the reference's single-threaded result; for mixed
 *     scenes the reference's result depends on thread interleaving.
 */
#define _GNU_SOURCE
#include "rt_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static __thread char g_err[512];
static void set_err(const char* msg, const char* arg) {
  snprintf(g_err, sizeof g_err, "%s%s%s", msg, arg ? ": " : "", arg ? arg : "");
}
const char* orc_last_error(void) { return g_err; }

/* ------------------------------------------------------------------------------------------------
 * Eigen 3.3.7 float expression order (Redux.h:96-110 halving unroller: size-3 sums are
 * x0 + (x1 + x2); Matrix4f*Vector4f packet product accumulates columns left to right;
 * OrthoMethods.h:43-47 cross; Dot.h:124-134 normalized divides by sqrt, returns input if |x|^2 <= 0)
 * ---------------------------------------------------------------------------------------------- */
static inline float e_dot(const float* a, const float* b) { return a[0] * b[0] + (a[1] * b[1] + a[2] * b[2]); }
static inline float e_sqnorm(const float* a) { return a[0] * a[0] + (a[1] * a[1] + a[2] * a[2]); }
static inline float e_norm(const float* a) { return sqrtf(e_sqnorm(a)); }
static inline void e_normalized(const float* a, float* o) {
  float z = e_sqnorm(a);
  if (z > 0.0f) {
    float r = sqrtf(z);
    o[0] = a[0] / r; o[1] = a[1] / r; o[2] = a[2] / r;
  } else {
    o[0] = a[0]; o[1] = a[1]; o[2] = a[2];
  }
}
static inline void e_cross(const float* a, const float* b, float* o) {
  float x = a[1] * b[2] - a[2] * b[1];
  float y = a[2] * b[0] - a[0] * b[2];
  float z = a[0] * b[1] - a[1] * b[0];
  o[0] = x; o[1] = y; o[2] = z;
}
static inline void e_sub(const float* a, const float* b, float* o) { o[0] = a[0] - b[0]; o[1] = a[1] - b[1]; o[2] = a[2] - b[2]; }
/* Matrix3f (column-major m[9]) * Vector3f: per row a0 + (a1 + a2) */
static inline void e_m3v3(const float* m, const float* v, float* o) {
  float r[3];
  for (int i = 0; i < 3; i++) r[i] = m[i] * v[0] + (m[3 + i] * v[1] + m[6 + i] * v[2]);
  o[0] = r[0]; o[1] = r[1]; o[2] = r[2];
}
/* Affine3f (column-major 4x4) * Vector3f = (T.matrix() * [v;1]).head<3>() (Transform.h:1372-1392) */
static inline void e_affv3(const float* m, const float* v, float* o) {
  float r[3];
  for (int i = 0; i < 3; i++) r[i] = ((m[i] * v[0] + m[4 + i] * v[1]) + m[8 + i] * v[2]) + m[12 + i];
  o[0] = r[0]; o[1] = r[1]; o[2] = r[2];
}
static inline void e_m4v4(const float* m, const float* v, float* o) {
  float r[4];
  for (int i = 0; i < 4; i++) r[i] = ((m[i] * v[0] + m[4 + i] * v[1]) + m[8 + i] * v[2]) + m[12 + i] * v[3];
  memcpy(o, r, 16);
}
/* Matrix3f::inverse (InverseImpl.h:124-171), m column-major */
static void e_m3inv(const float* m, float* o) {
#define M_(i, j) m[(j) * 3 + (i)]
#define COF(i, j) (M_(((i) + 1) % 3, ((j) + 1) % 3) * M_(((i) + 2) % 3, ((j) + 2) % 3) - \
                   M_(((i) + 1) % 3, ((j) + 2) % 3) * M_(((i) + 2) % 3, ((j) + 1) % 3))
  float c0[3] = {COF(0, 0), COF(1, 0), COF(2, 0)};
  float det = c0[0] * M_(0, 0) + (c0[1] * M_(1, 0) + c0[2] * M_(2, 0));
  float invdet = 1.0f / det;
  float r[9];
  /* result.row(0) = cofactors_col0 * invdet */
  r[0 * 3 + 0] = c0[0] * invdet; r[1 * 3 + 0] = c0[1] * invdet; r[2 * 3 + 0] = c0[2] * invdet;
  r[0 * 3 + 1] = COF(0, 1) * invdet; r[1 * 3 + 1] = COF(1, 1) * invdet; r[2 * 3 + 1] = COF(2, 1) * invdet;
  r[0 * 3 + 2] = COF(0, 2) * invdet; r[1 * 3 + 2] = COF(1, 2) * invdet; r[2 * 3 + 2] = COF(2, 2) * invdet;
#undef COF
#undef M_
  memcpy(o, r, 36);
}
/* Affine3f::inverse(Affine) (Transform.h:1202-1229) */
static void e_affinv(const float* t, float* o) {
  float L[9], Li[9], tr[3], r[16];
  for (int j = 0; j < 3; j++) for (int i = 0; i < 3; i++) L[j * 3 + i] = t[j * 4 + i];
  e_m3inv(L, Li);
  tr[0] = t[12]; tr[1] = t[13]; tr[2] = t[14];
  float lt[3];
  e_m3v3(Li, tr, lt);
  for (int j = 0; j < 3; j++) for (int i = 0; i < 3; i++) r[j * 4 + i] = Li[j * 3 + i];
  r[12] = -lt[0]; r[13] = -lt[1]; r[14] = -lt[2];
  r[3] = r[7] = r[11] = 0.0f; r[15] = 1.0f;
  memcpy(o, r, 64);
}
/* Matrix3f * Matrix3f lazy product: element (i,j) = row_i . col_j reduced a0 + (a1 + a2) */
static void e_m3m3(const float* a, const float* b, float* o) {
  float r[9];
  for (int j = 0; j < 3; j++)
    for (int i = 0; i < 3; i++)
      r[j * 3 + i] = a[i] * b[j * 3 + 0] + (a[3 + i] * b[j * 3 + 1] + a[6 + i] * b[j * 3 + 2]);
  memcpy(o, r, 36);
}
/* Affine * Affine (Transform.h:1481-1495) */
static void e_affmul(const float* a, const float* b, float* o) {
  float La[9], Lb[9], Lr[9], tb[3], ta[3], tr[3], r[16];
  for (int j = 0; j < 3; j++) for (int i = 0; i < 3; i++) { La[j * 3 + i] = a[j * 4 + i]; Lb[j * 3 + i] = b[j * 4 + i]; }
  e_m3m3(La, Lb, Lr);
  tb[0] = b[12]; tb[1] = b[13]; tb[2] = b[14]; ta[0] = a[12]; ta[1] = a[13]; ta[2] = a[14];
  e_m3v3(La, tb, tr);
  for (int j = 0; j < 3; j++) for (int i = 0; i < 3; i++) r[j * 4 + i] = Lr[j * 3 + i];
  r[12] = tr[0] + ta[0]; r[13] = tr[1] + ta[1]; r[14] = tr[2] + ta[2];
  r[3] = r[7] = r[11] = 0.0f; r[15] = 1.0f;
  memcpy(o, r, 64);
}
static void e_identity(float* m) { memset(m, 0, 64); m[0] = m[5] = m[10] = m[15] = 1.0f; }
/* Transform::scale(float) : linearExt() *= s (Transform.h:857-862) */
static void e_scale(float* m, float s) { for (int j = 0; j < 3; j++) for (int i = 0; i < 3; i++) m[j * 4 + i] *= s; }
/* Transform::translate(v): translationExt() += linearExt() * v (Transform.h:898-903) */
static void e_translate(float* m, const float* v) {
  float L[9], lv[3];
  for (int j = 0; j < 3; j++) for (int i = 0; i < 3; i++) L[j * 3 + i] = m[j * 4 + i];
  e_m3v3(L, v, lv);
  m[12] += lv[0]; m[13] += lv[1]; m[14] += lv[2];
}
/* std::min / std::max (bits/stl_algobase.h): min(a,b) = b<a ? b : a ; max(a,b) = a<b ? b : a */
static inline float s_min(float a, float b) { return (b < a) ? b : a; }
static inline float s_max(float a, float b) { return (a < b) ? b : a; }

/* ------------------------------------------------------------------------------------------------
 * Mesh (Tucano::Mesh + Face semantics)
 * ---------------------------------------------------------------------------------------------- */
typedef struct {
  float ka[3], kd[3], ks[3];
  float ns, ni, d;
  char name[256];
} omat;

struct orc_mesh {
  int32_t nv, nf, nm;
  float* v;    /* [nv][4] object space, w = 1   (Mesh::vertices) */
  float* vn;   /* [nv][3] (Mesh::normals) */
  uint32_t* f; /* [nf][3] */
  float* fn;   /* [nf][3] Face::normal */
  int32_t* fm; /* [nf] Face::material_id */
  omat* mats;
  float scale;      /* normalization_scale */
  float center[3];  /* objectCenter */
  float M[16];      /* getShapeModelMatrix() */
  /* hoisted loop invariants (same float expressions, evaluated once) */
  float* wv;   /* [nv][3] M * v           (flyscene.cpp:449,574-576) */
  float* nn;   /* [nv][3] normals[i].normalized()   (flyscene.cpp:599) */
  float* fnn;  /* [nf][3] face.normal.normalized()  (flyscene.cpp:450,577) */
  float* fdist;/* [nf] facenormal.dot(vert0)         (flyscene.cpp:459) */
  float Minv[16]; /* getShapeModelMatrix().inverse() (flyscene.cpp:486) */
  float MS[9];    /* its linear block (flyscene.cpp:487) */
};

static void mat_default(omat* m) {
  /* Tucano::Material::Mtl defaults (tucano/materials/mtl.hpp:22-40) */
  memset(m, 0, sizeof *m);
  m->ka[0] = m->ka[1] = m->ka[2] = 0.3f;
  m->kd[0] = m->kd[1] = m->kd[2] = 0.5f;
  m->ks[0] = m->ks[1] = m->ks[2] = 1.0f;
  m->ns = 10.0f; m->ni = 0.0f; m->d = 1.0f;
}

typedef struct { char* p; size_t n, cap; } sbuf;
typedef struct { void* p; size_t n, cap, esz; } vec;
static int vec_push(vec* v, const void* e) {
  if (v->n == v->cap) {
    size_t nc = v->cap ? v->cap * 2 : 64;
    void* np = realloc(v->p, nc * v->esz);
    if (!np) return -1;
    v->p = np; v->cap = nc;
  }
  memcpy((char*)v->p + v->n * v->esz, e, v->esz);
  v->n++;
  return 0;
}

/* getline(in, line): returns malloc'd line without '\n' (keeps '\r'), NULL at EOF */
static char* read_line(FILE* f, sbuf* b) {
  int c; b->n = 0;
  int any = 0;
  while ((c = fgetc(f)) != EOF) {
    any = 1;
    if (c == '\n') break;
    if (b->n + 2 > b->cap) { b->cap = b->cap ? b->cap * 2 : 256; b->p = (char*)realloc(b->p, b->cap); }
    b->p[b->n++] = (char)c;
  }
  if (!any) return NULL;
  if (b->n + 1 > b->cap) { b->cap = b->cap ? b->cap * 2 : 256; b->p = (char*)realloc(b->p, b->cap); }
  b->p[b->n] = 0;
  return b->p;
}
static void strip_crlf(char* s) {
  char* w = s;
  for (char* r = s; *r; r++) if (*r != '\n' && *r != '\r') *w++ = *r;
  *w = 0;
}
/* getPathName (objimporter.hpp:44-48 / mtlIO.hpp:36-40) */
static void path_of(const char* fn, char* out, size_t cap) {
  const char* a = strrchr(fn, '/');
  const char* b = strrchr(fn, '\\');
  const char* l = a > b ? a : b;
  size_t n = l ? (size_t)(l - fn) + 1 : 0;
  if (n >= cap) n = cap - 1;
  memcpy(out, fn, n); out[n] = 0;
}

/* MaterialImporter::loadMTL (mtlIO.hpp:49-140) */
static int load_mtl(vec* mats, const char* filename) {
  FILE* f = fopen(filename, "rb");
  if (!f) return -1;
  sbuf b = {0};
  char* line;
  while ((line = read_line(f, &b))) {
    if (!line[0]) continue;
    /* tokens split on single ' ' (std::getline(ss, s, ' ')) */
    char* toks[16]; int nt = 0;
    char* p = line;
    for (;;) {
      char* sp = strchr(p, ' ');
      if (nt < 16) toks[nt++] = p;
      if (!sp) break;
      *sp = 0; p = sp + 1;
      if (!*p) break; /* getline at EOF after delimiter yields no further token */
    }
    if (nt == 0) continue;
    omat* cur = mats->n ? &((omat*)mats->p)[mats->n - 1] : NULL;
    if (!strcmp(toks[0], "#")) continue;
    if (!strcmp(toks[0], "newmtl")) {
      omat m; mat_default(&m);
      if (nt > 1) { strncpy(m.name, toks[1], sizeof m.name - 1); strip_crlf(m.name); }
      vec_push(mats, &m);
    } else if (!cur) {
      continue; /* reference: UB (materials.back() on empty); ignored */
    } else if (!strcmp(toks[0], "Ns") && nt > 1) {
      cur->ns = (float)atof(toks[1]);
    } else if (!strcmp(toks[0], "Ka") && nt > 3) {
      cur->ka[0] = (float)atof(toks[1]); cur->ka[1] = (float)atof(toks[2]); cur->ka[2] = (float)atof(toks[3]);
    } else if (!strcmp(toks[0], "Kd") && nt > 3) {
      cur->kd[0] = (float)atof(toks[1]); cur->kd[1] = (float)atof(toks[2]); cur->kd[2] = (float)atof(toks[3]);
    } else if (!strcmp(toks[0], "Ks") && nt > 3) {
      cur->ks[0] = (float)atof(toks[1]); cur->ks[1] = (float)atof(toks[2]); cur->ks[2] = (float)atof(toks[3]);
    } else if (!strcmp(toks[0], "Ni") && nt > 1) {
      cur->ni = (float)atof(toks[1]);
    } else if (!strcmp(toks[0], "d") && nt > 1) {
      cur->d = (float)atof(toks[1]);
    }
  }
  free(b.p);
  fclose(f);
  if (mats->n == 0) { omat m; mat_default(&m); vec_push(mats, &m); }
  return 0;
}

/* istringstream >> float x3 (libstdc++ num_get -> strtof on the numeric prefix) */
static int parse_floats(const char* s, float* out, int n) {
  char* end;
  for (int k = 0; k < n; k++) {
    while (*s == ' ' || *s == '\t' || *s == '\r' || *s == '\f' || *s == '\v') s++;
    out[k] = strtof(s, &end);
    if (end == s) return k;
    s = end;
  }
  return n;
}

static void mesh_free_arrays(orc_mesh* m) {
  free(m->v); free(m->vn); free(m->f); free(m->fn); free(m->fm); free(m->mats);
  free(m->wv); free(m->nn); free(m->fnn); free(m->fdist);
}
void orc_mesh_free(orc_mesh* m) { if (m) { mesh_free_arrays(m); free(m); } }

/* Mesh::loadVertices bounding box / scale / centre (mesh.hpp:592-628) */
static void mesh_load_vertices(orc_mesh* m) {
  m->scale = 1.0f; m->center[0] = m->center[1] = m->center[2] = 0.0f;
  if (m->nv == 0) return;
  float xMax = m->v[0], xMin = m->v[0], yMax = m->v[1], yMin = m->v[1], zMax = m->v[2], zMin = m->v[2];
  for (int32_t i = 0; i < m->nv; i++) {
    const float* v = &m->v[4 * i];
    xMax = s_max(v[0], xMax); yMax = s_max(v[1], yMax); zMax = s_max(v[2], zMax);
    xMin = s_min(v[0], xMin); yMin = s_min(v[1], yMin); zMin = s_min(v[2], zMin);
  }
  float ext = s_max(s_max(fabsf(xMax - xMin), fabsf(yMax - yMin)), fabsf(zMax - zMin));
  m->scale = (float)(1.0 / (double)ext);
  m->center[0] = (float)((double)(xMax + xMin) / 2.0);
  m->center[1] = (float)((double)(yMax + yMin) / 2.0);
  m->center[2] = (float)((double)(zMax + zMin) / 2.0);
}

/* computeNormals (objimporter.hpp:81-106) over the index groups */
static void compute_normals(orc_mesh* m, int32_t ng, const int32_t* gcount, const uint32_t* idx) {
  memset(m->vn, 0, sizeof(float) * 3 * (size_t)m->nv);
  size_t off = 0;
  for (int32_t g = 0; g < ng; g++) {
    for (int32_t i = 0; i + 2 < gcount[g]; i += 3) {
      const uint32_t* t = &idx[off + i];
      const float *p0 = &m->v[4 * t[0]], *p1 = &m->v[4 * t[1]], *p2 = &m->v[4 * t[2]];
      float a[3], b[3], v0[3], v1[3], c[3], n[3];
      e_sub(p1, p0, a); e_normalized(a, v0);
      e_sub(p2, p0, b); e_normalized(b, v1);
      e_cross(v0, v1, c); e_normalized(c, n);
      for (int k = 0; k < 3; k++) {
        float* d = &m->vn[3 * t[k]];
        d[0] = d[0] + n[0]; d[1] = d[1] + n[1]; d[2] = d[2] + n[2];
      }
    }
    off += (size_t)gcount[g];
  }
  for (int32_t i = 0; i < m->nv; i++) {
    float* d = &m->vn[3 * i];
    e_normalized(d, d); /* normalize(): in place, unchanged if |d|^2 <= 0 */
  }
}

/* the model-matrix-dependent data: getShapeModelMatrix() = modelMatrix * shapeMatrix (model.hpp:102-105)
 * with shapeMatrix from normalizeModelMatrix (model.hpp:169-173), its inverse, the world vertices and the
 * plane distances (hoisted from calculateDistance, flyscene.cpp:444-478) */
static void mesh_place(orc_mesh* m, const float* model) {
  float shape[16], negc[3] = {-m->center[0], -m->center[1], -m->center[2]};
  e_identity(shape); e_scale(shape, m->scale); e_translate(shape, negc);
  e_affmul(model, shape, m->M);
  e_affinv(m->M, m->Minv);
  for (int j = 0; j < 3; j++) for (int i = 0; i < 3; i++) m->MS[j * 3 + i] = m->Minv[j * 4 + i];
  for (int32_t i = 0; i < m->nv; i++) e_affv3(m->M, &m->v[4 * i], &m->wv[3 * i]);
  for (int32_t f = 0; f < m->nf; f++) m->fdist[f] = e_dot(&m->fnn[3 * f], &m->wv[3 * m->f[3 * f]]);
}

/* derived per-mesh data: shape-model matrix, hoisted invariants */
static int mesh_finish(orc_mesh* m) {
  float model[16];
  e_identity(model);  /* Model::modelMatrix as loaded: identity */
  m->wv = (float*)malloc(sizeof(float) * 3 * (size_t)(m->nv ? m->nv : 1));
  m->nn = (float*)malloc(sizeof(float) * 3 * (size_t)(m->nv ? m->nv : 1));
  m->fnn = (float*)malloc(sizeof(float) * 3 * (size_t)(m->nf ? m->nf : 1));
  m->fdist = (float*)malloc(sizeof(float) * (size_t)(m->nf ? m->nf : 1));
  if (!m->wv || !m->nn || !m->fnn || !m->fdist) { set_err("out of memory", NULL); return -1; }
  for (int32_t i = 0; i < m->nv; i++) e_normalized(&m->vn[3 * i], &m->nn[3 * i]);
  for (int32_t f = 0; f < m->nf; f++) e_normalized(&m->fn[3 * f], &m->fnn[3 * f]);
  mesh_place(m, model);
  return 0;
}

/* Model::modelMatrix set by the caller (model.hpp: an Affine3f the application may rotate / scale; the
 * face normals stay the loaded object-space ones, as in the reference, whose calculateDistance uses
 * getFace().normal against world vertices). model16: column-major 4x4 affine. Build scenes afterwards. */
void orc_mesh_set_model(orc_mesh* m, const float* model16) { mesh_place(m, model16); }

/* createFaces (mesh.hpp:448-482) + common tail of loadObjFile (objimporter.hpp:284-336) */
static int mesh_build(orc_mesh* m, int32_t ng, const int32_t* gcount, const uint32_t* idx,
                      const int32_t* gmat, int have_vn) {
  mesh_load_vertices(m);
  if (!have_vn) compute_normals(m, ng, gcount, idx);
  int64_t nf = 0;
  for (int32_t g = 0; g < ng; g++) {
    if (gcount[g] % 3 != 0) { set_err("index group not a multiple of 3 (reference reads out of bounds)", NULL); return -1; }
    nf += gcount[g] / 3;
  }
  m->nf = (int32_t)nf;
  m->f = (uint32_t*)malloc(sizeof(uint32_t) * 3 * (size_t)(nf ? nf : 1));
  m->fn = (float*)malloc(sizeof(float) * 3 * (size_t)(nf ? nf : 1));
  m->fm = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nf ? nf : 1));
  if (!m->f || !m->fn || !m->fm) { set_err("out of memory", NULL); return -1; }
  size_t off = 0, fi = 0;
  for (int32_t g = 0; g < ng; g++) {
    for (int32_t i = 0; i < gcount[g]; i += 3, fi++) {
      const uint32_t* t = &idx[off + i];
      for (int k = 0; k < 3; k++) {
        if (t[k] >= (uint32_t)m->nv) { set_err("face index out of range", NULL); return -1; }
        m->f[3 * fi + k] = t[k];
      }
      m->fm[fi] = gmat[g];
      const float *p0 = &m->v[4 * t[0]], *p1 = &m->v[4 * t[1]], *p2 = &m->v[4 * t[2]];
      float a[3], b[3], v0[3], v1[3], c[3];
      e_sub(p2, p0, a); e_normalized(a, v1);
      e_sub(p1, p0, b); e_normalized(b, v0);
      e_cross(v0, v1, c); e_normalized(c, &m->fn[3 * fi]);
    }
    off += (size_t)gcount[g];
  }
  return mesh_finish(m);
}

int orc_mesh_load_obj(const char* path, orc_mesh** out) {
  *out = NULL;
  FILE* f = fopen(path, "rb");
  if (!f) { set_err("Cannot open", path); return -1; }
  char dir[4096]; path_of(path, dir, sizeof dir);
  vec verts = {0, 0, 0, sizeof(float) * 4}, norms = {0, 0, 0, sizeof(float) * 3};
  vec idx = {0, 0, 0, sizeof(uint32_t)}, gcount = {0, 0, 0, sizeof(int32_t)}, gmat = {0, 0, 0, sizeof(int32_t)};
  vec mats = {0, 0, 0, sizeof(omat)};
  int32_t zero = 0, minus1 = -1, current_mat = -1;
  vec_push(&gcount, &zero); vec_push(&gmat, &minus1);
  sbuf b = {0};
  char* line;
  int rc = 0;
  while ((line = read_line(f, &b))) {
    size_t L = strlen(line);
    int32_t* gc = &((int32_t*)gcount.p)[gcount.n - 1];
    if (!strncmp(line, "mtllib", 6)) {
      if (L < 7) { set_err("malformed mtllib line", NULL); rc = -1; break; }
      char fn[8192]; snprintf(fn, sizeof fn, "%s%s", dir, line + 7); strip_crlf(fn);
      load_mtl(&mats, fn);
    } else if (!strncmp(line, "usemtl", 6)) {
      if (*gc != 0) { vec_push(&gcount, &zero); vec_push(&gmat, &minus1); }
      if (L < 7) { set_err("malformed usemtl line", NULL); rc = -1; break; }
      char nm[4096]; snprintf(nm, sizeof nm, "%s", line + 7); strip_crlf(nm);
      for (size_t i = 0; i < mats.n; i++)
        if (!strcmp(((omat*)mats.p)[i].name, nm)) current_mat = (int32_t)i;
      ((int32_t*)gmat.p)[gmat.n - 1] = current_mat;
    } else if (L >= 2 && line[0] == 'v' && line[1] == ' ') {
      float v[4] = {0, 0, 0, 1.0f};
      parse_floats(line + 2, v, 3);
      vec_push(&verts, v);
    } else if (L >= 2 && line[0] == 'v' && line[1] == 'n') {
      float n[3] = {0, 0, 0};
      if (L >= 3) parse_floats(line + 3, n, 3);
      vec_push(&norms, n);
    } else if (L >= 2 && line[0] == 'v' && line[1] == 't') {
      /* texture coordinates: not used by the ray tracer */
    } else if (L >= 2 && line[0] == 'f' && line[1] == ' ') {
      char* p = line + 2;
      for (;;) {
        while (*p == ' ' || *p == '\t' || *p == '\r' || *p == '\v' || *p == '\f') p++;
        if (!*p) break;
        char* e = p;
        while (*e && *e != ' ' && *e != '\t' && *e != '\r' && *e != '\v' && *e != '\f') e++;
        long vid = strtol(p, NULL, 10); /* stoi(element before first '/') */
        uint32_t u = (uint32_t)(vid - 1);
        vec_push(&idx, &u);
        ((int32_t*)gcount.p)[gcount.n - 1]++;
        p = e;
      }
    }
  }
  free(b.p);
  fclose(f);
  if (rc) goto fail;
  orc_mesh* m = (orc_mesh*)calloc(1, sizeof *m);
  m->nv = (int32_t)verts.n;
  m->v = (float*)verts.p; verts.p = NULL;
  m->vn = (float*)malloc(sizeof(float) * 3 * (verts.n ? verts.n : 1));
  int have_vn = (norms.n == (size_t)m->nv);
  if (have_vn) memcpy(m->vn, norms.p, sizeof(float) * 3 * norms.n);
  m->nm = (int32_t)mats.n;
  m->mats = (omat*)mats.p; mats.p = NULL;
  /* only non-empty index groups become index buffers (objimporter.hpp:312-319) */
  int32_t ng = 0;
  int32_t* gc2 = (int32_t*)malloc(sizeof(int32_t) * gcount.n);
  int32_t* gm2 = (int32_t*)malloc(sizeof(int32_t) * gcount.n);
  for (size_t g = 0; g < gcount.n; g++)
    if (((int32_t*)gcount.p)[g] > 0) { gc2[ng] = ((int32_t*)gcount.p)[g]; gm2[ng] = ((int32_t*)gmat.p)[g]; ng++; }
  rc = (m->nv > 0) ? mesh_build(m, ng, gc2, (uint32_t*)idx.p, gm2, have_vn) : 0;
  if (m->nv == 0) { m->f = NULL; m->nf = 0; mesh_finish(m); }
  free(gc2); free(gm2);
  free(norms.p); free(idx.p); free(gcount.p); free(gmat.p);
  if (rc) { orc_mesh_free(m); return rc; }
  *out = m;
  return 0;
fail:
  free(verts.p); free(norms.p); free(idx.p); free(gcount.p); free(gmat.p); free(mats.p);
  return rc;
}

int orc_mesh_from_arrays(int32_t nv, const float* v3, const float* vn3, int32_t ng, const int32_t* gcount,
                         const uint32_t* idx, const int32_t* gmat, int32_t nm, const float* mat12,
                         orc_mesh** out) {
  *out = NULL;
  orc_mesh* m = (orc_mesh*)calloc(1, sizeof *m);
  m->nv = nv;
  m->v = (float*)malloc(sizeof(float) * 4 * (size_t)(nv ? nv : 1));
  m->vn = (float*)malloc(sizeof(float) * 3 * (size_t)(nv ? nv : 1));
  for (int32_t i = 0; i < nv; i++) {
    m->v[4 * i] = v3[3 * i]; m->v[4 * i + 1] = v3[3 * i + 1]; m->v[4 * i + 2] = v3[3 * i + 2]; m->v[4 * i + 3] = 1.0f;
  }
  if (vn3) memcpy(m->vn, vn3, sizeof(float) * 3 * (size_t)nv);
  m->nm = nm;
  m->mats = (omat*)calloc((size_t)(nm ? nm : 1), sizeof(omat));
  for (int32_t i = 0; i < nm; i++) {
    const float* p = &mat12[12 * i];
    omat* o = &m->mats[i];
    memcpy(o->ka, p, 12); memcpy(o->kd, p + 3, 12); memcpy(o->ks, p + 6, 12);
    o->ns = p[9]; o->ni = p[10]; o->d = p[11];
    snprintf(o->name, sizeof o->name, "material_%d", i);
  }
  int rc = mesh_build(m, ng, gcount, idx, gmat, vn3 != NULL);
  if (rc) { orc_mesh_free(m); return rc; }
  *out = m;
  return 0;
}

void orc_mesh_counts(const orc_mesh* m, int32_t* nv, int32_t* nf, int32_t* nm) {
  if (nv) *nv = m->nv;
  if (nf) *nf = m->nf;
  if (nm) *nm = m->nm;
}

void orc_mesh_export(const orc_mesh* m, float* v4, float* vn3, uint32_t* fidx, float* fn3, int32_t* fmat,
                     float* mats, float* M16, float* sc4) {
  if (v4) memcpy(v4, m->v, sizeof(float) * 4 * (size_t)m->nv);
  if (vn3) memcpy(vn3, m->vn, sizeof(float) * 3 * (size_t)m->nv);
  if (fidx) memcpy(fidx, m->f, sizeof(uint32_t) * 3 * (size_t)m->nf);
  if (fn3) memcpy(fn3, m->fn, sizeof(float) * 3 * (size_t)m->nf);
  if (fmat) memcpy(fmat, m->fm, sizeof(int32_t) * (size_t)m->nf);
  if (mats)
    for (int32_t i = 0; i < m->nm; i++) {
      float* p = &mats[12 * i];
      memcpy(p, m->mats[i].ka, 12); memcpy(p + 3, m->mats[i].kd, 12); memcpy(p + 6, m->mats[i].ks, 12);
      p[9] = m->mats[i].ns; p[10] = m->mats[i].ni; p[11] = m->mats[i].d;
    }
  if (M16) memcpy(M16, m->M, 64);
  if (sc4) { sc4[0] = m->scale; sc4[1] = m->center[0]; sc4[2] = m->center[1]; sc4[3] = m->center[2]; }
}

/* ------------------------------------------------------------------------------------------------
 * Synthetic soup (build-defined workload for C3/C4; not a reference function)
 * ---------------------------------------------------------------------------------------------- */
static inline uint64_t splitmix64(uint64_t* s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static inline float u01(uint64_t* s) { return (float)(splitmix64(s) >> 40) * (1.0f / 16777216.0f); }
void orc_generate_soup(int32_t n, uint64_t seed, float* v) {
  uint64_t s = seed;
  for (int32_t t = 0; t < n; t++) {
    float c[3];
    for (int k = 0; k < 3; k++) c[k] = u01(&s) - 0.5f;
    for (int j = 0; j < 3; j++)
      for (int k = 0; k < 3; k++) {
        float off = (u01(&s) * 2.0f - 1.0f) * 0.01f;
        v[9 * (size_t)t + 3 * j + k] = c[k] + off;
      }
  }
}

/* ------------------------------------------------------------------------------------------------
 * Flat box partition (src/BoundingBox.cpp, src/flyscene.cpp:399-428)
 * ---------------------------------------------------------------------------------------------- */
typedef struct {
  float low[3], high[3], shape[3];
  int failed[3];
  int32_t* faces; int32_t n, cap;
} obox;

/* Per-face record in reference iteration order (box creation order, then in-box order): the inputs
 * calculateDistance reads for one face, stored contiguously so a ray streams through them. Data
 * placement only: every value is the same float the indexed arrays hold (fnn, fdist, wv). */
typedef struct {
  float fn[3], fd;
  float w0[3], w1[3], w2[3];
  int32_t f;
} ofrec;

struct orc_scene {
  orc_mesh* m;
  obox* boxes; int32_t nb, cap;
  int32_t* pass_counts; int32_t npass;
  /* trace layout (built once after the partition): box bounds as structure-of-arrays for the
   * vectorised intersectBox sweep, face records in iteration order, boff[b] = first record of box b */
  float* bsoa;   /* [6][nb]: low x, low y, low z, high x, high y, high z */
  int32_t* boff; /* [nb + 1] */
  ofrec* fr;     /* [nf] */
};

static void box_reshape(obox* b) { for (int k = 0; k < 3; k++) b->shape[k] = b->high[k] - b->low[k]; } /* BoundingBox.cpp:18-24 */

/* BoundingBox::hasFace / hasVertex (BoundingBox.cpp:26-39) */
static int box_has_face(const obox* b, const orc_mesh* m, int32_t f) {
  for (int k = 0; k < 3; k++) {
    const float* v = &m->v[4 * m->f[3 * f + k]];
    if (!(v[0] >= b->low[0] && v[0] <= b->high[0] && v[1] >= b->low[1] && v[1] <= b->high[1] &&
          v[2] >= b->low[2] && v[2] <= b->high[2]))
      return 0;
  }
  return 1;
}

/* BoundingBox::fitFaces (BoundingBox.cpp:48-90) */
static void box_fit(obox* b, const orc_mesh* m) {
  if (b->n <= 0) return;
  const float* t = &m->v[4 * m->f[3 * b->faces[0]]];
  float minx = t[0], maxx = t[0], miny = t[1], maxy = t[1], minz = t[2], maxz = t[2];
  for (int32_t i = 0; i < b->n; i++) {
    for (int j = 0; j < 3; j++) {
      const float* v = &m->v[4 * m->f[3 * b->faces[i] + j]];
      float x = v[0], y = v[1], z = v[2];
      if (x < minx) minx = x; else if (x > maxx) maxx = x;
      if (y < miny) miny = y; else if (y > maxy) maxy = y;
      if (z < minz) minz = z; else if (z > maxz) maxz = z;
    }
  }
  b->low[0] = minx; b->low[1] = miny; b->low[2] = minz;
  b->high[0] = maxx; b->high[1] = maxy; b->high[2] = maxz;
  box_reshape(b);
}

/* BoundingBox::averageVertexCoord (BoundingBox.cpp:151-161) */
static float box_average(const obox* b, const orc_mesh* m, int axis) {
  float avg = 0.0f;
  for (int32_t i = 0; i < b->n; i++) {
    const uint32_t* f = &m->f[3 * b->faces[i]];
    avg += m->v[4 * f[0] + axis];
    avg += m->v[4 * f[1] + axis];
    avg += m->v[4 * f[2] + axis];
  }
  avg /= (float)((size_t)b->n * 3);
  return avg;
}

static obox* scene_new_box(orc_scene* s) {
  if (s->nb == s->cap) {
    s->cap = s->cap ? s->cap * 2 : 16;
    s->boxes = (obox*)realloc(s->boxes, sizeof(obox) * (size_t)s->cap);
  }
  obox* b = &s->boxes[s->nb++];
  memset(b, 0, sizeof *b);
  return b;
}

/* BoundingBox::splitBox (BoundingBox.cpp:109-149). returns: 1 = new box created, 0 = failed axis
 * (returned `this`), -1 = all axes failed (returned nullptr) */
static int box_split(orc_scene* s, int32_t bi) {
  const orc_mesh* m = s->m;
  obox* b = &s->boxes[bi];
  float oldLow[3], oldHigh[3];
  memcpy(oldLow, b->low, 12); memcpy(oldHigh, b->high, 12);
  float w = b->shape[0], h = b->shape[1], d = b->shape[2];
  int choice;
  if ((w >= h || b->failed[1]) && (w >= d || b->failed[2]) && !b->failed[0]) choice = 0;
  else if ((h >= w || b->failed[0]) && (h >= d || b->failed[2]) && !b->failed[1]) choice = 1;
  else if (!(b->failed[0] && b->failed[1] && b->failed[2])) choice = 2;
  else return -1;
  b->high[choice] = box_average(b, m, choice);
  box_reshape(b);
  /* outsideFaces (BoundingBox.cpp:92-107): stable partition */
  int32_t* in = (int32_t*)malloc(sizeof(int32_t) * (size_t)(b->n ? b->n : 1));
  int32_t* outf = (int32_t*)malloc(sizeof(int32_t) * (size_t)(b->n ? b->n : 1));
  int32_t nin = 0, nout = 0;
  for (int32_t i = 0; i < b->n; i++) {
    int32_t f = b->faces[i];
    if (!box_has_face(b, m, f)) outf[nout++] = f; else in[nin++] = f;
  }
  if (nin == 0 || nout == 0) {
    if (nin == 0) { free(in); in = outf; nin = nout; outf = NULL; }
    else free(outf);
    free(b->faces); b->faces = in; b->n = nin; b->cap = nin;
    b->failed[choice] = 1;
    memcpy(b->low, oldLow, 12); memcpy(b->high, oldHigh, 12);
    box_reshape(b);
    return 0;
  }
  free(b->faces); b->faces = in; b->n = nin; b->cap = nin;
  b->failed[0] = b->failed[1] = b->failed[2] = 0;
  obox* nbx = scene_new_box(s); /* may realloc: re-fetch b */
  b = &s->boxes[bi];
  nbx->faces = outf; nbx->n = nout; nbx->cap = nout;
  box_fit(nbx, m);
  box_fit(b, m);
  return 1;
}

static void scene_trace_layout(orc_scene* s) {
  const orc_mesh* m = s->m;
  const int32_t nb = s->nb;
  s->bsoa = (float*)malloc(sizeof(float) * 6 * (size_t)(nb ? nb : 1));
  s->boff = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nb + 1));
  s->fr = (ofrec*)malloc(sizeof(ofrec) * (size_t)(m->nf ? m->nf : 1));
  int32_t off = 0;
  for (int32_t b = 0; b < nb; b++) {
    const obox* bx = &s->boxes[b];
    for (int k = 0; k < 3; k++) {
      s->bsoa[(size_t)k * nb + b] = bx->low[k];
      s->bsoa[(size_t)(3 + k) * nb + b] = bx->high[k];
    }
    s->boff[b] = off;
    for (int32_t i = 0; i < bx->n; i++) {
      const int32_t f = bx->faces[i];
      const uint32_t* id = &m->f[3 * (size_t)f];
      ofrec* r = &s->fr[off++];
      memcpy(r->fn, &m->fnn[3 * (size_t)f], 12);
      r->fd = m->fdist[f];
      memcpy(r->w0, &m->wv[3 * (size_t)id[0]], 12);
      memcpy(r->w1, &m->wv[3 * (size_t)id[1]], 12);
      memcpy(r->w2, &m->wv[3 * (size_t)id[2]], 12);
      r->f = f;
    }
  }
  s->boff[nb] = off;
}

int orc_scene_build(orc_mesh* m, int32_t min_faces, int32_t max_boxes, orc_scene** out) {
  orc_scene* s = (orc_scene*)calloc(1, sizeof *s);
  s->m = m;
  int32_t pcap = 64;
  s->pass_counts = (int32_t*)malloc(sizeof(int32_t) * (size_t)pcap);
  /* generateBoundingBoxes (flyscene.cpp:399-420): BoundingBox(true) + fitMesh */
  obox* b0 = scene_new_box(s);
  b0->n = b0->cap = m->nf;
  b0->faces = (int32_t*)malloc(sizeof(int32_t) * (size_t)(m->nf ? m->nf : 1));
  for (int32_t i = 0; i < m->nf; i++) b0->faces[i] = i;
  box_fit(b0, m);
  int notDone = 1;
  while (notDone && s->nb < max_boxes) {
    notDone = 0;
    int32_t ncur = s->nb; /* vector<BoundingBox*> current = boxes */
    if (s->npass == pcap) { pcap *= 2; s->pass_counts = (int32_t*)realloc(s->pass_counts, sizeof(int32_t) * (size_t)pcap); }
    s->pass_counts[s->npass++] = ncur;
    for (int32_t bi = 0; bi < ncur; bi++) {
      obox* b = &s->boxes[bi];
      if (b->n > min_faces && (!b->failed[0] || !b->failed[1] || !b->failed[2])) {
        int r = box_split(s, bi);
        while (r == 0) r = box_split(s, bi);
        notDone = 1;
      }
    }
  }
  scene_trace_layout(s);
  *out = s;
  return 0;
}

void orc_scene_free(orc_scene* s) {
  if (!s) return;
  for (int32_t i = 0; i < s->nb; i++) free(s->boxes[i].faces);
  free(s->boxes); free(s->pass_counts);
  free(s->bsoa); free(s->boff); free(s->fr);
  free(s);
}
int32_t orc_scene_box_count(const orc_scene* s) { return s->nb; }
void orc_scene_boxes(const orc_scene* s, float* bounds6, int32_t* counts, int32_t* face_order) {
  size_t off = 0;
  for (int32_t i = 0; i < s->nb; i++) {
    const obox* b = &s->boxes[i];
    if (bounds6) { memcpy(&bounds6[6 * i], b->low, 12); memcpy(&bounds6[6 * i + 3], b->high, 12); }
    if (counts) counts[i] = b->n;
    if (face_order) memcpy(&face_order[off], b->faces, sizeof(int32_t) * (size_t)b->n);
    off += (size_t)b->n;
  }
}
int32_t orc_scene_pass_counts(const orc_scene* s, int32_t* out, int32_t max) {
  for (int32_t i = 0; i < s->npass && i < max; i++) out[i] = s->pass_counts[i];
  return s->npass;
}

/* ------------------------------------------------------------------------------------------------
 * Camera (tucano/camera.hpp, tucano/utils/flycamera.hpp)
 * ---------------------------------------------------------------------------------------------- */
void orc_camera_flycam(int32_t W, int32_t H, float dx, float dy, float dz, orc_camera* c) {
  /* Flycamera::translate (flycamera.hpp:196-202): translation_vector += yaw * (-dx,-dy,dz) * speed,
   * yaw = AngleAxisf(0, UnitY) -> identity rotation matrix */
  float I9[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
  float v[3] = {-dx, -dy, dz}, yv[3], tv[3];
  const float speed = 0.05f; /* flycamera.hpp:107 */
  e_m3v3(I9, v, yv);
  tv[0] = 0.0f + yv[0] * speed; tv[1] = 0.0f + yv[1] * speed; tv[2] = 0.0f + yv[2] * speed;
  /* updateViewMatrix (flycamera.hpp:166-191) with rotation_X/Y = 0: rotate(I), rotate(I),
   * translate(default_translation (0,0,-2)), translate(translation_vector) */
  float view[16], deft[3] = {0.0f, 0.0f, -2.0f};
  e_identity(view);
  e_translate(view, deft);
  e_translate(view, tv);
  memcpy(c->view, view, 64);
  /* setPerspectiveMatrix(60, w/(float)h, ..), setViewport (flyscene.cpp:14-15) */
  c->viewport[0] = 0.0f; c->viewport[1] = 0.0f; c->viewport[2] = (float)W; c->viewport[3] = (float)H;
  c->fovy = 60.0f;
  c->aspect = (float)W / (float)H;
}

/* traceRayThread ray generation (flyscene.cpp:301,308): o = getCenter(), d = N(screenToWorld(i,j) - o) */
void orc_camera_ray(const orc_camera* c, int32_t i, int32_t j, float* o, float* d) {
  /* getCenter (camera.hpp:115-118): view.linear().inverse() * (-view.translation()) */
  float L[9], Li[9], nt[3];
  for (int b = 0; b < 3; b++) for (int a = 0; a < 3; a++) L[b * 3 + a] = c->view[b * 4 + a];
  e_m3inv(L, Li);
  nt[0] = -c->view[12]; nt[1] = -c->view[13]; nt[2] = -c->view[14];
  e_m3v3(Li, nt, o);
  /* screenToWorld (camera.hpp:155-173, getPerspectiveScale :263-266) */
  float rx = (float)i, ry = (float)j;
  float nc[3];
  nc[0] = (float)(2.0 * (double)(rx - c->viewport[0]) / (double)c->viewport[2] - 1.0);
  nc[1] = (float)(1.0 - 2.0 * (double)(ry - c->viewport[1]) / (double)c->viewport[3]);
  nc[2] = -1.0f;
  float persp = (float)((double)1.0f / tan((double)(c->fovy / 2.0f) * (M_PI / 180.0)));
  float scale = (float)(1.0 / (double)persp);
  nc[0] *= c->aspect * scale;
  nc[1] *= scale;
  float vinv[16], w[3], diff[3];
  e_affinv(c->view, vinv);
  e_affv3(vinv, nc, w);
  e_sub(w, o, diff);
  e_normalized(diff, d);
}

/* ------------------------------------------------------------------------------------------------
 * Tracing (src/flyscene.cpp)
 * ---------------------------------------------------------------------------------------------- */
typedef struct { float ka[3], kd[3], ks[3], shininess; } mstate; /* Flyscene members hpp:179-182 */

typedef struct {
  orc_scene* s;
  const float* lights; int32_t nl;
  const orc_render_opts* opt;
} tctx;

/* per-ray object-space transform hoisted out of intersectBox (flyscene.cpp:485-490) */
typedef struct { float o2[3], d2[3]; } oray;
static void obj_ray(const orc_mesh* m, const float* o, const float* d, oray* r) {
  float t[3];
  e_affv3(m->Minv, o, r->o2);
  e_m3v3(m->MS, d, t);
  e_normalized(t, r->d2);
}
/* intersectBox (flyscene.cpp:484-507) */
static int intersect_box(const oray* r, const obox* b) {
  float tmin[3], tmax[3], tin3[3], tout3[3];
  for (int k = 0; k < 3; k++) {
    tmin[k] = (b->low[k] - r->o2[k]) / r->d2[k];
    tmax[k] = (b->high[k] - r->o2[k]) / r->d2[k];
    tin3[k] = s_min(tmin[k], tmax[k]);
    tout3[k] = s_max(tmin[k], tmax[k]);
  }
  float tin = s_max(tin3[0], s_max(tin3[1], tin3[2]));
  float tout = s_min(tout3[0], s_min(tout3[1], tout3[2]));
  return !(tin > tout || tout < 0);
}

/* intersectBox for boxes [b0, b0+n) of the flat list: acc[i] = intersectBox(box b0+i). The same
 * expressions as intersect_box per box, over the structure-of-arrays bounds so that the compiler
 * vectorises the sweep (IEEE division and compares are exact in SIMD lanes; s_min/s_max map to
 * minps/maxps with the operand order that keeps std::min/max's NaN behaviour). */
__attribute__((target_clones("avx2", "default")))
static void intersect_boxes(const orc_scene* s, const oray* r, int32_t b0, int32_t n, uint8_t* acc) {
  const int32_t nb = s->nb;
  const float *lx = s->bsoa + b0, *ly = s->bsoa + (size_t)nb + b0, *lz = s->bsoa + 2 * (size_t)nb + b0;
  const float *hx = s->bsoa + 3 * (size_t)nb + b0, *hy = s->bsoa + 4 * (size_t)nb + b0, *hz = s->bsoa + 5 * (size_t)nb + b0;
  const float ox = r->o2[0], oy = r->o2[1], oz = r->o2[2], dx = r->d2[0], dy = r->d2[1], dz = r->d2[2];
  for (int32_t i = 0; i < n; i++) {
    const float ax = (lx[i] - ox) / dx, bx = (hx[i] - ox) / dx;
    const float ay = (ly[i] - oy) / dy, by = (hy[i] - oy) / dy;
    const float az = (lz[i] - oz) / dz, bz = (hz[i] - oz) / dz;
    const float tin = s_max(s_min(ax, bx), s_max(s_min(ay, by), s_min(az, bz)));
    const float tout = s_min(s_max(ax, bx), s_min(s_max(ay, by), s_max(az, bz)));
    acc[i] = (uint8_t)!(tin > tout || tout < 0);
  }
}

/* interpolateNormal (flyscene.cpp:572-600) for face f with world vertices v0..v2 and unit face normal fn */
static void interpolate_normal_v(const orc_mesh* m, int32_t f, const float* v0, const float* v1, const float* v2,
                                 const float* fn, const float* P, float* out) {
  const uint32_t* id = &m->f[3 * f];
  float e0[3], e1[3], e2[3], i0[3], i1[3], i2[3], a0[3], a1[3], a2[3];
  e_sub(v1, v0, e0); e_sub(v2, v1, e1); e_sub(v0, v2, e2);
  e_sub(P, v0, i0); e_sub(P, v1, i1); e_sub(P, v2, i2);
  e_cross(e0, i0, a0); e_cross(e1, i1, a1); e_cross(e2, i2, a2);
  if (e_dot(fn, a0) < 0 || e_dot(fn, a1) < 0 || e_dot(fn, a2) < 0) { out[0] = out[1] = out[2] = 0.0f; return; }
  float area0 = e_norm(a0) / 2, area1 = e_norm(a1) / 2, area2 = e_norm(a2) / 2;
  float ne2[3] = {-e2[0], -e2[1], -e2[2]}, c[3];
  e_cross(e0, ne2, c);
  float area = e_norm(c) / 2;
  const float *n0 = &m->nn[3 * id[0]], *n1 = &m->nn[3 * id[1]], *n2 = &m->nn[3 * id[2]];
  float s[3];
  for (int k = 0; k < 3; k++) s[k] = (n0[k] * area1 / area + n1[k] * area2 / area) + n2[k] * area0 / area;
  e_normalized(s, out);
}
static void interpolate_normal(const orc_mesh* m, int32_t f, const float* P, float* out) {
  const uint32_t* id = &m->f[3 * f];
  interpolate_normal_v(m, f, &m->wv[3 * id[0]], &m->wv[3 * id[1]], &m->wv[3 * id[2]], &m->fnn[3 * f], P, out);
}

/* calculateDistance (flyscene.cpp:444-478): returns t (or -1), P */
static float calc_distance(const orc_mesh* m, const float* o, const float* d, int32_t f, float* P) {
  const float* fn = &m->fnn[3 * f];
  if (e_dot(fn, d) == 0) return -1.0f;
  float orth = m->fdist[f] - e_dot(o, fn);
  float t = orth / e_dot(d, fn);
  float p[3] = {o[0] + t * d[0], o[1] + t * d[1], o[2] + t * d[2]};
  float n[3];
  interpolate_normal(m, f, p, n);
  if (e_norm(n) == 0) return -1.0f;
  if (P) memcpy(P, p, 12);
  return t;
}

/* calculateDistance on an iteration-order face record (same arithmetic as calc_distance) */
static inline float calc_distance_rec(const orc_mesh* m, const ofrec* fr, const float* o, const float* d, float* P) {
  if (e_dot(fr->fn, d) == 0) return -1.0f;
  float orth = fr->fd - e_dot(o, fr->fn);
  float t = orth / e_dot(d, fr->fn);
  float p[3] = {o[0] + t * d[0], o[1] + t * d[1], o[2] + t * d[2]};
  /* interpolateNormal's inside test first (its early return, flyscene.cpp:584-586); the rest of it
   * only for points that pass */
  float e0[3], e1[3], e2[3], i0[3], i1[3], i2[3], a0[3], a1[3], a2[3];
  e_sub(fr->w1, fr->w0, e0); e_sub(fr->w2, fr->w1, e1); e_sub(fr->w0, fr->w2, e2);
  e_sub(p, fr->w0, i0); e_sub(p, fr->w1, i1); e_sub(p, fr->w2, i2);
  e_cross(e0, i0, a0); e_cross(e1, i1, a1); e_cross(e2, i2, a2);
  if (e_dot(fr->fn, a0) < 0 || e_dot(fr->fn, a1) < 0 || e_dot(fr->fn, a2) < 0) return -1.0f;
  float n[3];
  interpolate_normal_v(m, fr->f, fr->w0, fr->w1, fr->w2, fr->fn, p, n);
  if (e_norm(n) == 0) return -1.0f;
  if (P) memcpy(P, p, 12);
  return t;
}

#define ORC_BOX_CHUNK 512

/* calculateMinimumFace (flyscene.cpp:373-396): boxes in creation order, faces in in-box order, the
 * first minimum kept (strict <) */
static int32_t closest(const orc_scene* s, const float* o, const float* d, float* tbest, float* Pbest) {
  const orc_mesh* m = s->m;
  oray r; obj_ray(m, o, d, &r);
  float best = INFINITY;
  int32_t bf = -1;
  float P[3] = {0, 0, 0}, Pc[3];
  uint8_t acc[ORC_BOX_CHUNK];
  for (int32_t b0 = 0; b0 < s->nb; b0 += ORC_BOX_CHUNK) {
    const int32_t n = s->nb - b0 < ORC_BOX_CHUNK ? s->nb - b0 : ORC_BOX_CHUNK;
    intersect_boxes(s, &r, b0, n, acc);
    for (int32_t i = 0; i < n; i++) {
      if (!acc[i]) continue;
      const int32_t bi = b0 + i;
      for (int32_t k = s->boff[bi]; k < s->boff[bi + 1]; k++) {
        float t = calc_distance_rec(m, &s->fr[k], o, d, Pc);
        if (0 <= t && t < best) { best = t; bf = s->fr[k].f; memcpy(P, Pc, 12); }
      }
    }
  }
  *tbest = best;
  if (Pbest) memcpy(Pbest, P, 12);
  return bf;
}

/* shadow (flyscene.cpp:510-526) */
static int shadow(const orc_scene* s, const float* P, const float* L) {
  const orc_mesh* m = s->m;
  float inter[3];
  for (int k = 0; k < 3; k++) inter[k] = P[k] + 0.003f * L[k];
  oray r; obj_ray(m, P, L, &r);
  uint8_t acc[ORC_BOX_CHUNK];
  for (int32_t b0 = 0; b0 < s->nb; b0 += ORC_BOX_CHUNK) {
    const int32_t n = s->nb - b0 < ORC_BOX_CHUNK ? s->nb - b0 : ORC_BOX_CHUNK;
    intersect_boxes(s, &r, b0, n, acc);
    for (int32_t i = 0; i < n; i++) {
      if (!acc[i]) continue;
      const int32_t bi = b0 + i;
      for (int32_t k = s->boff[bi]; k < s->boff[bi + 1]; k++)
        if (calc_distance_rec(m, &s->fr[k], inter, L, NULL) >= 0) return 1;
    }
  }
  return 0;
}

/* calcSingleColor (flyscene.cpp:542-566) */
static void calc_single(const tctx* c, mstate* st, int32_t f, const float* o, const float* L, const float* I,
                        const float* P, float* out) {
  const orc_mesh* m = c->s->m;
  if (c->opt->shadows && shadow(c->s, P, L)) { out[0] = out[1] = out[2] = 0.0f; return; }
  if (m->fm[f] != -1) {
    const omat* mt = &m->mats[m->fm[f]];
    memcpy(st->ka, mt->ka, 12); memcpy(st->kd, mt->kd, 12); memcpy(st->ks, mt->ks, 12);
    st->shininess = mt->ns;
  }
  float n[3], R[3], E[3], oe[3];
  interpolate_normal(m, f, P, n);
  float nl2 = 2 * e_dot(n, L);
  for (int k = 0; k < 3; k++) R[k] = L[k] - nl2 * n[k];
  e_sub(o, P, oe); e_normalized(oe, E);
  float dif = s_max(e_dot(L, n), 0.f);
  float spe = s_max(powf(e_dot(R, E), st->shininess), 0.f);
  for (int k = 0; k < 3; k++) {
    float amb = I[k] * st->ka[k];
    float di = (I[k] * st->kd[k]) * dif;
    float sp = (I[k] * st->ks[k]) * spe;
    out[k] = (amb + di) + sp;
  }
}

/* calculateColor (flyscene.cpp:603-614) */
static void calc_color(const tctx* c, mstate* st, int32_t f, const float* o, const float* P, float* out) {
  float sum[3] = {0.0f, 0.0f, 0.0f};
  for (int32_t l = 0; l < c->nl; l++) {
    const float* lp = &c->lights[6 * l];
    float diff[3], nd[3], L[3], col[3];
    e_sub(P, lp, diff); e_normalized(diff, nd);
    L[0] = -nd[0]; L[1] = -nd[1]; L[2] = -nd[2];
    calc_single(c, st, f, o, L, lp + 3, P, col);
    sum[0] += col[0]; sum[1] += col[1]; sum[2] += col[2];
  }
  /* directional lights: the stored vector is the light direction as is (flyscene.cpp:610-612) */
  for (int32_t l = 0; l < c->opt->n_dir_lights; l++) {
    const float* dl = &c->opt->dir_lights6[6 * l];
    float L[3] = {dl[0], dl[1], dl[2]}, col[3];
    calc_single(c, st, f, o, L, dl + 3, P, col);
    sum[0] += col[0]; sum[1] += col[1]; sum[2] += col[2];
  }
  for (int k = 0; k < 3; k++) out[k] = s_max(s_min(sum[k], 1.f), 0.f);
}

/* traceRay (flyscene.cpp:317-371) */
static void trace_ray(const tctx* c, mstate* st, const float* o, const float* d, int depth, float* out,
                      int32_t* face0, float* t0) {
  const orc_mesh* m = c->s->m;
  if (depth == c->opt->max_depth) { out[0] = out[1] = out[2] = 0.0f; return; }
  float t, P[3];
  int32_t f = closest(c->s, o, d, &t, P);
  if (face0) { *face0 = f; *t0 = t; }
  if (t == INFINITY) {
    if (depth == 0) memcpy(out, c->opt->background, 12);
    else out[0] = out[1] = out[2] = 0.0f;
    return;
  }
  if (c->opt->box_colors3) {
    /* RENDER_BOUNDINGBOX_COLORED_TRIANGLES (flyscene.cpp:334-348): color += box->color over every box
     * (creation order) with box->hasFace(minimum_face); `number` stays 0, so the sum is returned as is */
    float col[3] = {0.0f, 0.0f, 0.0f};
    for (int32_t b = 0; b < c->s->nb; b++)
      if (box_has_face(&c->s->boxes[b], m, f))
        for (int k = 0; k < 3; k++) col[k] += c->opt->box_colors3[3 * (size_t)b + k];
    memcpy(out, col, 12);
    return;
  }
  float direct[3];
  calc_color(c, st, f, o, P, direct);
  if (m->fm[f] != -1) memcpy(st->ks, m->mats[m->fm[f]].ks, 12);
  float dn[3], n[3], r[3], off[3], rc[3];
  e_normalized(d, dn);
  interpolate_normal(m, f, P, n);
  /* reflect (flyscene.cpp:480-482): (d - 2*(d.dot(n)*n)).normalized() */
  float dd = e_dot(dn, n), tmp[3];
  for (int k = 0; k < 3; k++) tmp[k] = dn[k] - 2 * (dd * n[k]);
  e_normalized(tmp, r);
  for (int k = 0; k < 3; k++) off[k] = P[k] + 0.001f * r[k];
  trace_ray(c, st, off, r, depth + 1, rc, NULL, NULL);
  for (int k = 0; k < 3; k++) {
    float c2 = direct[k] + rc[k] * st->ks[k];
    out[k] = s_max(s_min(c2, 1.f), 0.f);
  }
}

void orc_render_opts_default(orc_render_opts* o, int32_t full) {
  memset(o, 0, sizeof *o);
  o->max_depth = full ? 2 : 1;
  o->shadows = full ? 1 : 0;
  o->background[0] = o->background[1] = o->background[2] = 0.9f; /* flyscene.hpp:175 */
  /* default material members (flyscene.hpp:179-182) */
  o->def_mat[0] = o->def_mat[1] = o->def_mat[2] = 0.2f;
  o->def_mat[3] = 0.9f; o->def_mat[4] = 0.9f; o->def_mat[5] = 0.0f;
  o->def_mat[6] = o->def_mat[7] = o->def_mat[8] = 0.0f;
  o->def_mat[9] = 0.0f;
}

typedef struct {
  tctx c;
  const orc_camera* cam;
  int32_t W, H, n, tid, nth;
  const int32_t* pix;
  float *rgb, *t; int32_t* face;
} job;

static void* render_worker(void* arg) {
  job* j = (job*)arg;
  float o[3], d[3];
  for (int32_t k = j->tid; k < j->n; k += j->nth) {
    int32_t pi, pj;
    if (j->pix) { pi = j->pix[2 * k]; pj = j->pix[2 * k + 1]; }
    else { pj = k / j->W; pi = k % j->W; }
    mstate st;
    memcpy(st.ka, j->c.opt->def_mat, 12); memcpy(st.kd, j->c.opt->def_mat + 3, 12);
    memcpy(st.ks, j->c.opt->def_mat + 6, 12); st.shininess = j->c.opt->def_mat[9];
    orc_camera_ray(j->cam, pi, pj, o, d);
    float col[3]; int32_t f = -1; float t = INFINITY;
    trace_ray(&j->c, &st, o, d, 0, col, &f, &t);
    if (j->rgb) memcpy(&j->rgb[3 * (size_t)k], col, 12);
    if (j->face) j->face[k] = f;
    if (j->t) j->t[k] = t;
  }
  return NULL;
}

int orc_render(orc_scene* s, const orc_camera* cam, const float* lights, int32_t nl, int32_t W, int32_t H,
               const orc_render_opts* opts, int32_t n_pixels, const int32_t* pixels, int32_t nthreads,
               float* rgb, int32_t* face, float* t) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  int32_t n = pixels ? n_pixels : W * H;
  /* rows interleaved across threads for full frames (deterministic: per-pixel state) */
  job jobs[256];
  pthread_t th[256];
  for (int32_t i = 0; i < nthreads; i++) {
    jobs[i].c.s = s; jobs[i].c.lights = lights; jobs[i].c.nl = nl; jobs[i].c.opt = opts;
    jobs[i].cam = cam; jobs[i].W = W; jobs[i].H = H; jobs[i].n = n; jobs[i].tid = i; jobs[i].nth = nthreads;
    jobs[i].pix = pixels; jobs[i].rgb = rgb; jobs[i].t = t; jobs[i].face = face;
  }
  if (nthreads == 1) { render_worker(&jobs[0]); return 0; }
  for (int32_t i = 0; i < nthreads; i++) pthread_create(&th[i], NULL, render_worker, &jobs[i]);
  for (int32_t i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
  return 0;
}

/* BoundingBox::setRandomColor (BoundingBox.cpp:163-165) per box in creation order, as the reference built
 * with g++ evaluates Vector3f(rand()/RAND_MAX, x3): arguments right to left, so a box's first rand() call
 * is its blue channel (pinned by tests/golden/boxcolor_kat.bin, oracle/boxcolor_kat.cpp) */
void orc_box_colors_glibc(int32_t n, float* out3) {
  srand(1);
  for (int32_t i = 0; i < n; i++) {
    const float c2 = rand() / (float)RAND_MAX, c1 = rand() / (float)RAND_MAX, c0 = rand() / (float)RAND_MAX;
    out3[3 * i] = c0; out3[3 * i + 1] = c1; out3[3 * i + 2] = c2;
  }
}

int orc_closest(orc_scene* s, int32_t n, const float* o, const float* d, int32_t* face, float* t, float* P) {
  for (int32_t i = 0; i < n; i++) {
    float tt, pp[3];
    int32_t f = closest(s, &o[3 * i], &d[3 * i], &tt, pp);
    face[i] = f; t[i] = tt;
    if (P) memcpy(&P[3 * i], pp, 12);
  }
  return 0;
}
int orc_shadow(orc_scene* s, int32_t n, const float* P, const float* L, int32_t* out) {
  for (int32_t i = 0; i < n; i++) out[i] = shadow(s, &P[3 * i], &L[3 * i]);
  return 0;
}

/* ------------------------------------------------------------------------------------------------
 * Primitive KAT entry (op codes: oracle/eigen_kat.cpp)
 * ---------------------------------------------------------------------------------------------- */
int orc_kat(int32_t op, int32_t n, const float* in, float* out) {
  for (int32_t k = 0; k < n; k++) {
    switch (op) {
      case 0: { const float* a = in + 6 * k; out[k] = e_dot(a, a + 3); break; }
      case 1: { e_normalized(in + 3 * k, out + 3 * k); break; }
      case 2: { const float* a = in + 6 * k; e_cross(a, a + 3, out + 3 * k); break; }
      case 3: { const float* a = in + 12 * k; e_m3v3(a, a + 9, out + 3 * k); break; }
      case 4: { const float* a = in + 19 * k; e_affv3(a, a + 16, out + 3 * k); break; }
      case 5: { const float* a = in + 20 * k; e_m4v4(a, a + 16, out + 4 * k); break; }
      case 6: { e_m3inv(in + 9 * k, out + 9 * k); break; }
      case 7: { e_affinv(in + 16 * k, out + 16 * k); break; }
      case 8: {
        const float* a = in + 4 * k;
        float sh[16], md[16], nc[3] = {-a[1], -a[2], -a[3]};
        e_identity(sh); e_scale(sh, a[0]); e_translate(sh, nc);
        e_identity(md); e_affmul(md, sh, out + 16 * k);
        break; }
      case 9: { const float* a = in + 6 * k; for (int i = 0; i < 3; i++) out[3 * k + i] = a[i] + 0.001f * a[3 + i]; break; }
      case 10: { const float* a = in + 6 * k; for (int i = 0; i < 3; i++) out[3 * k + i] = a[i] + 0.003f * a[3 + i]; break; }
      case 11: {
        const float* a = in + 6 * k; float dd = e_dot(a, a + 3), t[3];
        for (int i = 0; i < 3; i++) t[i] = a[i] - 2 * (dd * a[3 + i]);
        e_normalized(t, out + 3 * k); break; }
      case 12: {
        const float* a = in + 6 * k; float nl2 = 2 * e_dot(a + 3, a);
        for (int i = 0; i < 3; i++) out[3 * k + i] = a[i] - nl2 * a[3 + i];
        break; }
      case 13: {
        const float* a = in + 13 * k; float n0[3], n1[3], n2[3], s[3];
        e_normalized(a, n0); e_normalized(a + 3, n1); e_normalized(a + 6, n2);
        float area0 = a[9], area1 = a[10], area2 = a[11], area = a[12];
        for (int i = 0; i < 3; i++) s[i] = (n0[i] * area1 / area + n1[i] * area2 / area) + n2[i] * area0 / area;
        e_normalized(s, out + 3 * k); break; }
      case 14: { out[k] = e_norm(in + 3 * k) / 2; break; }
      case 15: {
        const float* a = in + 16 * k; float L[9], Li[9], nt[3];
        for (int j = 0; j < 3; j++) for (int i = 0; i < 3; i++) L[j * 3 + i] = a[j * 4 + i];
        e_m3inv(L, Li); nt[0] = -a[12]; nt[1] = -a[13]; nt[2] = -a[14];
        e_m3v3(Li, nt, out + 3 * k); break; }
      case 16: {
        const float* a = in + 24 * k;
        float nc[3];
        nc[0] = (float)(2.0 * (double)(a[16] - a[18]) / (double)a[20] - 1.0);
        nc[1] = (float)(1.0 - 2.0 * (double)(a[17] - a[19]) / (double)a[21]);
        nc[2] = -1.0f;
        float persp = (float)((double)1.0f / tan((double)(a[22] / 2.0f) * (M_PI / 180.0)));
        float scale = (float)(1.0 / (double)persp);
        nc[0] *= a[23] * scale; nc[1] *= scale;
        float vinv[16]; e_affinv(a, vinv); e_affv3(vinv, nc, out + 3 * k); break; }
      default: set_err("unknown kat op", NULL); return -1;
    }
  }
  return 0;
}
