/*
 * accel.c -- host build of the device scene image: flattened triangle
 * records, pre-normalised normals, materials, lights and the octree.
 *
 * Flattening:
 *   prim p = global triangle index in (object, LIFO triangle) order, the
 *   lexicographic tie-break key of cpu/hit.c:59,82; e1 = v1-v0, e2 = v2-v0
 *   are the exact subtractions of cpu/hit.c:16-17; vertex normals are
 *   normalised once with the reference's own vector3_normalize
 *   (cpu/hit.c:11-13 does it per test: same bits).
 *
 * Octree (replaces gpu/partitioning/octree.cu:362-411 create_octree, whose
 * object-level "deepest cell fully containing the AABB" rule leaves straddlers
 * at the root): every node splits its cell at the
 * centre into 8 octants; a triangle *reference* goes to every octant its
 * (exact, SAT) triangle/box test overlaps; leaves stop at RT_OCT_LEAF
 * references or depth RT_OCT_DEPTH or when splitting stops separating.
 * Node boxes are the union of the full bounding boxes of the triangles below
 * them (not clipped to the cell): a ray that the reference's float
 * Moller-Trumbore test accepts for triangle T passes within the device's
 * per-ray epsilon of bbox(T), hence through every ancestor box of every leaf
 * holding T, so culling can never drop the reference's winner
 * (DESIGN.md "Conservative culling").
 * Children of a node are stored contiguously; triangle records of a leaf are
 * stored contiguously (duplicated per leaf), so a leaf visit streams whole
 * 48-byte records.
 */
#define _GNU_SOURCE
#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "rt_cull.h"
#include "rt_internal.h"

#define RT_OCT_LEAF 4
#define RT_OCT_DEPTH 20
/* size_stop >= 1 disables the "triangles larger than the cell" stop (the
 * SAH and RT_OCT_LEAF_CAP below decide instead) */
#define RT_OCT_SIZE_STOP 4.0

static float u2f(uint32_t u)
{
  float f;
  memcpy(&f, &u, 4);
  return f;
}

/* ---------------------------------------------------------------- octree */

typedef struct { double lo[3], hi[3]; } dbox;

typedef struct {
  const float *rec;        /* prim-order records (12 floats each) */
  const float *pbox;       /* prim bounding boxes, 6 floats each  */
  double pad;              /* conservative slack of the overlap tests */
  double size_stop;        /* leaf once mean triangle extent > size_stop * cell */
  int leaf_max;            /* leaf at <= leaf_max references */
  double c_box;            /* SAH cost of a child box test (triangle test = 1) */
  int leaf_cap;            /* split past this many references while it separates them */
} oct_input;

/* One (sub)tree under construction.  Node slot 0 is its root. */
typedef struct {
  float *node; size_t nnode, node_cap;
  uint32_t *refs; size_t nref, ref_cap;
  size_t leaves, max_depth, max_leaf;
  int oom;
} oct_tree;

/* A subtree deferred to the worker threads: node `slot` of the top tree. */
typedef struct {
  size_t slot;
  dbox cell;
  uint32_t *ids;
  size_t n, depth;
  oct_tree sub;
} oct_task;

typedef struct {
  oct_task *t;
  size_t n, cap;
  int oom;
} oct_tasks;

static int ensure(void **p, size_t *cap, size_t need, size_t elem)
{
  if (need <= *cap)
    return 0;
  size_t nc = *cap ? *cap : 1024;
  while (nc < need)
    nc *= 2;
  void *np = realloc(*p, nc * elem);
  if (!np)
    return -1;
  *p = np;
  *cap = nc;
  return 0;
}

/* Triangle/box overlap by the separating axis theorem (13 axes), in double,
 * against the box grown by `pad` -- conservative: never says "no" for a
 * triangle that touches the box. */
static int tri_box_overlap(const float *rec, const dbox *b, double pad)
{
  double c[3], h[3], v[3][3];
  for (int i = 0; i < 3; i++)
  {
    c[i] = 0.5 * (b->lo[i] + b->hi[i]);
    h[i] = 0.5 * (b->hi[i] - b->lo[i]) + pad;
  }
  /* record layout: q0 = v0.xyz e1.x, q1 = e1.yz e2.xy, q2 = e2.z ... */
  double v0[3] = { rec[0], rec[1], rec[2] };
  double e1[3] = { rec[3], rec[4], rec[5] };
  double e2[3] = { rec[6], rec[7], rec[8] };
  for (int i = 0; i < 3; i++)
  {
    v[0][i] = v0[i] - c[i];
    v[1][i] = v0[i] + e1[i] - c[i];
    v[2][i] = v0[i] + e2[i] - c[i];
  }
  for (int i = 0; i < 3; i++)
  {
    double mn = fmin(v[0][i], fmin(v[1][i], v[2][i]));
    double mx = fmax(v[0][i], fmax(v[1][i], v[2][i]));
    if (mn > h[i] || mx < -h[i])
      return 0;
  }
  double f[3][3];
  for (int i = 0; i < 3; i++)
  {
    f[0][i] = v[1][i] - v[0][i];
    f[1][i] = v[2][i] - v[1][i];
    f[2][i] = v[0][i] - v[2][i];
  }
  double n[3] = { f[0][1] * f[1][2] - f[0][2] * f[1][1], f[0][2] * f[1][0] - f[0][0] * f[1][2],
                  f[0][0] * f[1][1] - f[0][1] * f[1][0] };
  {
    double d = n[0] * v[0][0] + n[1] * v[0][1] + n[2] * v[0][2];
    double r = h[0] * fabs(n[0]) + h[1] * fabs(n[1]) + h[2] * fabs(n[2]);
    double slack = 1e-9 * (fabs(d) + r);
    if (d > r + slack || d < -r - slack)
      return 0;
  }
  for (int k = 0; k < 3; k++)
    for (int j = 0; j < 3; j++)
    {
      /* axis = unit_k x f_j */
      double a[3];
      int k1 = (k + 1) % 3, k2 = (k + 2) % 3;
      a[k] = 0;
      a[k1] = -f[j][k2];
      a[k2] = f[j][k1];
      double p0 = a[0] * v[0][0] + a[1] * v[0][1] + a[2] * v[0][2];
      double p1 = a[0] * v[1][0] + a[1] * v[1][1] + a[2] * v[1][2];
      double p2 = a[0] * v[2][0] + a[1] * v[2][1] + a[2] * v[2][2];
      double mn = fmin(p0, fmin(p1, p2)), mx = fmax(p0, fmax(p1, p2));
      double r = h[0] * fabs(a[0]) + h[1] * fabs(a[1]) + h[2] * fabs(a[2]);
      double slack = 1e-9 * (fabs(mn) + fabs(mx) + r);
      if (mn > r + slack || mx < -r - slack)
        return 0;
    }
  return 1;
}

static void write_node(float *nd, const float lo[3], const float hi[3], uint32_t first,
                       uint32_t count)
{
  nd[0] = lo[0];
  nd[1] = lo[1];
  nd[2] = lo[2];
  nd[3] = u2f(first);
  nd[4] = hi[0];
  nd[5] = hi[1];
  nd[6] = hi[2];
  nd[7] = u2f(count);
}

static void refs_box(const oct_input *in, const uint32_t *ids, size_t n, float lo[3], float hi[3],
                     double cell_ext, double *mean_ext)
{
  double sum = 0;
  for (int a = 0; a < 3; a++)
  {
    lo[a] = FLT_MAX;
    hi[a] = -FLT_MAX;
  }
  for (size_t i = 0; i < n; i++)
  {
    const float *pb = in->pbox + 6 * (size_t)ids[i];
    double e = 0;
    for (int a = 0; a < 3; a++)
    {
      if (pb[a] < lo[a]) lo[a] = pb[a];
      if (pb[3 + a] > hi[a]) hi[a] = pb[3 + a];
      e = fmax(e, (double)pb[3 + a] - pb[a]);
    }
    sum += fmin(e, cell_ext);
  }
  *mean_ext = n ? sum / (double)n : 0;
}

/* Subdivision stops at RT_OCT_LEAF references, at RT_OCT_DEPTH, once the
 * cell is much smaller than the triangles in it (size_stop), or when the
 * surface-area heuristic says the split does not pay: a visit of this node
 * tests its children's boxes (c_box each) and then the references of every
 * child the ray enters, with probability area(child box) / area(node box),
 * against testing all n references here (cost 1 each). */
#define RT_OCT_C_BOX 4.0
#define RT_OCT_LEAF_CAP 32
#define RT_OCT_MAX_SHRINK 40

static double box_area(const float lo[3], const float hi[3])
{
  double dx = (double)hi[0] - lo[0], dy = (double)hi[1] - lo[1], dz = (double)hi[2] - lo[2];
  if (dx < 0 || dy < 0 || dz < 0)
    return 0;
  return 2.0 * (dx * dy + dy * dz + dz * dx);
}

/* union of the references' boxes clipped to `cell` (rounded outwards) */
static void clip_to_cell(float lo[3], float hi[3], const dbox *cell)
{
  for (int a = 0; a < 3; a++)
  {
    float cl = (float)cell->lo[a], ch = (float)cell->hi[a];
    if ((double)cl > cell->lo[a]) cl = nextafterf(cl, -INFINITY);
    if ((double)ch < cell->hi[a]) ch = nextafterf(ch, INFINITY);
    if (lo[a] < cl) lo[a] = cl;
    if (hi[a] > ch) hi[a] = ch;
  }
}

static void build_node(const oct_input *in, oct_tree *b, size_t slot, const dbox *cell0,
                       uint32_t *ids, size_t n, size_t depth, oct_tasks *defer,
                       size_t defer_depth)
{
  if (b->oom)
    return;
  dbox cur = *cell0;
  const dbox *cell = &cur;
  int shrinks = 0;
tighten:;
  double cell_ext = cell->hi[0] - cell->lo[0];
  double mean_ext;
  float lo[3], hi[3];
  refs_box(in, ids, n, lo, hi, cell_ext, &mean_ext);
  /* clip to the cell: boxes of disjoint cells stay disjoint, so
   * front-to-back culling stops early */
  clip_to_cell(lo, hi, cell);
  if (depth > b->max_depth)
    b->max_depth = depth;
  int make_leaf = n <= (size_t)in->leaf_max || depth >= RT_OCT_DEPTH ||
                  mean_ext > in->size_stop * cell_ext;
  uint32_t *child_ids[8] = { 0 };
  size_t child_n[8] = { 0 };
  dbox cb[8];
  if (!make_leaf)
  {
    double mid[3];
    for (int a = 0; a < 3; a++)
      mid[a] = 0.5 * (cell->lo[a] + cell->hi[a]);
    double split_cost = 0, parent_area = box_area(lo, hi);
    for (int o = 0; o < 8 && !b->oom; o++)
    {
      for (int a = 0; a < 3; a++)
      {
        int upper = (o >> a) & 1;
        cb[o].lo[a] = upper ? mid[a] : cell->lo[a];
        cb[o].hi[a] = upper ? cell->hi[a] : mid[a];
      }
      child_ids[o] = malloc((n ? n : 1) * sizeof(uint32_t));
      if (!child_ids[o])
      {
        b->oom = 1;
        break;
      }
      for (size_t i = 0; i < n; i++)
      {
        const float *pb = in->pbox + 6 * (size_t)ids[i];
        int out = 0;
        for (int a = 0; a < 3; a++)
          out |= pb[a] > cb[o].hi[a] + in->pad || pb[3 + a] < cb[o].lo[a] - in->pad;
        if (out)
          continue;
        if (tri_box_overlap(in->rec + RT_TRI_FLOATS * (size_t)ids[i], &cb[o], in->pad))
          child_ids[o][child_n[o]++] = ids[i];
      }
      if (child_n[o])
      {
        float clo[3], chi[3];
        double unused;
        refs_box(in, child_ids[o], child_n[o], clo, chi, cell_ext, &unused);
        clip_to_cell(clo, chi, &cb[o]);
        double pr = parent_area > 0 ? box_area(clo, chi) / parent_area : 1.0;
        split_cost += in->c_box + (pr > 1 ? 1 : pr) * (double)child_n[o];
      }
    }
    int nonempty = 0, only = -1;
    for (int o = 0; o < 8; o++)
      if (child_n[o])
      {
        nonempty++;
        only = o;
      }
    if (!b->oom && nonempty == 1 && shrinks < RT_OCT_MAX_SHRINK)
    {
      /* everything lies in one octant: shrink this node's cell to it
       * instead of emitting a one-child node, and decide again */
      cur = cb[only];
      shrinks++;
      for (int o = 0; o < 8; o++)
      {
        free(child_ids[o]);
        child_ids[o] = NULL;
        child_n[o] = 0;
      }
      goto tighten;
    }
    /* SAH says "leaf" -- but a big leaf stalls a whole wave on one lane, so
     * above leaf_cap references always split (down to RT_OCT_DEPTH) */
    if (!b->oom && split_cost >= (double)n && n <= (size_t)in->leaf_cap)
      make_leaf = 1;
  }
  if (b->oom)
    goto done;
  if (make_leaf)
  {
    if (ensure((void **)&b->refs, &b->ref_cap, b->nref + n, sizeof(uint32_t)))
    {
      b->oom = 1;
      goto done;
    }
    memcpy(b->refs + b->nref, ids, n * sizeof(uint32_t));
    write_node(b->node + RT_NODE_FLOATS * slot, lo, hi, (uint32_t)b->nref,
               RT_NODE_LEAF | (uint32_t)n);
    b->nref += n;
    b->leaves++;
    if (n > b->max_leaf)
      b->max_leaf = n;
    goto done;
  }
  {
    int nc = 0;
    uint32_t omask = 0;
    for (int o = 0; o < 8; o++)
      if (child_n[o])
      {
        nc++;
        omask |= 1u << o;
      }
    size_t first = b->nnode;
    if (ensure((void **)&b->node, &b->node_cap, b->nnode + (size_t)nc,
               RT_NODE_FLOATS * sizeof(float)))
    {
      b->oom = 1;
      goto done;
    }
    b->nnode += (size_t)nc;
    write_node(b->node + RT_NODE_FLOATS * slot, lo, hi, (uint32_t)first,
               (uint32_t)nc | omask << 8);
    size_t k = 0;
    for (int o = 0; o < 8; o++)
    {
      if (!child_n[o])
        continue;
      if (defer && depth + 1 >= defer_depth)
      {
        /* hand the subtree to a worker; it owns child_ids[o] from now on */
        if (ensure((void **)&defer->t, &defer->cap, defer->n + 1, sizeof(oct_task)))
        {
          b->oom = 1;
          goto done;
        }
        oct_task *t = &defer->t[defer->n++];
        memset(t, 0, sizeof *t);
        t->slot = first + k;
        t->cell = cb[o];
        t->ids = child_ids[o];
        t->n = child_n[o];
        t->depth = depth + 1;
        child_ids[o] = NULL;
      }
      else
      {
        build_node(in, b, first + k, &cb[o], child_ids[o], child_n[o], depth + 1, defer,
                   defer_depth);
        free(child_ids[o]);
        child_ids[o] = NULL;
      }
      k++;
    }
  }
done:
  for (int o = 0; o < 8; o++)
    free(child_ids[o]);
}

typedef struct {
  const oct_input *in;
  oct_tasks *tasks;
  size_t next;
  pthread_mutex_t lock;
} oct_pool;

static void *oct_worker(void *arg)
{
  oct_pool *pool = arg;
  for (;;)
  {
    pthread_mutex_lock(&pool->lock);
    size_t i = pool->next++;
    pthread_mutex_unlock(&pool->lock);
    if (i >= pool->tasks->n)
      break;
    oct_task *t = &pool->tasks->t[i];
    if (ensure((void **)&t->sub.node, &t->sub.node_cap, 1, RT_NODE_FLOATS * sizeof(float)))
    {
      t->sub.oom = 1;
      continue;
    }
    t->sub.nnode = 1;
    build_node(pool->in, &t->sub, 0, &t->cell, t->ids, t->n, t->depth, NULL, 0);
    free(t->ids);
    t->ids = NULL;
  }
  return NULL;
}

/* Builds the octree of `ntri` prims: the top levels serially, the subtrees
 * below RT_OCT_PAR_DEPTH on worker threads, then splices the subtrees into
 * the top tree (children stay contiguous, leaf records contiguous). */
#define RT_OCT_PAR_DEPTH 2

static int build_octree(const oct_input *in, size_t ntri, const dbox *root, oct_tree *out)
{
  memset(out, 0, sizeof *out);
  oct_tasks tasks = { 0 };
  uint32_t *ids = malloc((ntri ? ntri : 1) * sizeof(uint32_t));
  if (!ids || ensure((void **)&out->node, &out->node_cap, 1, RT_NODE_FLOATS * sizeof(float)))
  {
    free(ids);
    return -1;
  }
  for (size_t i = 0; i < ntri; i++)
    ids[i] = (uint32_t)i;
  out->nnode = 1;
  build_node(in, out, 0, root, ids, ntri, 0, &tasks, RT_OCT_PAR_DEPTH);
  free(ids);

  int nthreads = (int)sysconf(_SC_NPROCESSORS_ONLN);
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 64) nthreads = 64;
  oct_pool pool = { in, &tasks, 0, PTHREAD_MUTEX_INITIALIZER };
  pthread_t tid[64];
  int started = 0;
  for (int t = 0; t < nthreads && (size_t)t < tasks.n; t++)
    if (pthread_create(&tid[t], NULL, oct_worker, &pool) == 0)
      started++;
  if (started == 0)
    oct_worker(&pool);
  for (int t = 0; t < started; t++)
    pthread_join(tid[t], NULL);

  /* splice: subtree local node i >= 1 -> out index base + i - 1 */
  for (size_t i = 0; i < tasks.n && !out->oom; i++)
  {
    oct_task *t = &tasks.t[i];
    oct_tree *sb = &t->sub;
    if (sb->oom)
    {
      out->oom = 1;
      break;
    }
    size_t nbase = out->nnode, rbase = out->nref;
    if (ensure((void **)&out->node, &out->node_cap, out->nnode + sb->nnode - 1,
               RT_NODE_FLOATS * sizeof(float)) ||
        ensure((void **)&out->refs, &out->ref_cap, out->nref + sb->nref, sizeof(uint32_t)))
    {
      out->oom = 1;
      break;
    }
    for (size_t k = 0; k < sb->nnode; k++)
    {
      float *dst = k == 0 ? out->node + RT_NODE_FLOATS * t->slot
                          : out->node + RT_NODE_FLOATS * (nbase + k - 1);
      const float *src = sb->node + RT_NODE_FLOATS * k;
      memcpy(dst, src, RT_NODE_FLOATS * sizeof(float));
      uint32_t first, cnt;
      memcpy(&first, &src[3], 4);
      memcpy(&cnt, &src[7], 4);
      first = (cnt & RT_NODE_LEAF) ? first + (uint32_t)rbase : first + (uint32_t)nbase - 1;
      dst[3] = u2f(first);
    }
    out->nnode += sb->nnode - 1;
    memcpy(out->refs + out->nref, sb->refs, sb->nref * sizeof(uint32_t));
    out->nref += sb->nref;
    out->leaves += sb->leaves;
    if (sb->max_depth > out->max_depth)
      out->max_depth = sb->max_depth;
    if (sb->max_leaf > out->max_leaf)
      out->max_leaf = sb->max_leaf;
  }
  for (size_t i = 0; i < tasks.n; i++)
  {
    free(tasks.t[i].ids);
    free(tasks.t[i].sub.node);
    free(tasks.t[i].sub.refs);
  }
  free(tasks.t);
  return out->oom ? -1 : 0;
}

/* -------------------------------------------------------------- flatten */

/* Squared distance from the origin to the triangle (a, b, c), in double
 * (closest point by Voronoi regions, Ericson, Real-Time Collision Detection
 * 5.1.5). */
static double origin_tri_dist2(const double a[3], const double b[3], const double c[3])
{
  double ab[3], ac[3], ap[3], bp[3], cp[3], q[3];
  for (int k = 0; k < 3; k++)
  {
    ab[k] = b[k] - a[k];
    ac[k] = c[k] - a[k];
    ap[k] = -a[k];
    bp[k] = -b[k];
    cp[k] = -c[k];
  }
#define DOT3(x, y) ((x)[0] * (y)[0] + (x)[1] * (y)[1] + (x)[2] * (y)[2])
  double d1 = DOT3(ab, ap), d2 = DOT3(ac, ap);
  if (d1 <= 0 && d2 <= 0)
    return DOT3(a, a);
  double d3 = DOT3(ab, bp), d4 = DOT3(ac, bp);
  if (d3 >= 0 && d4 <= d3)
    return DOT3(b, b);
  double vc = d1 * d4 - d3 * d2;
  if (vc <= 0 && d1 >= 0 && d3 <= 0)
  {
    double v = d1 / (d1 - d3);
    for (int k = 0; k < 3; k++) q[k] = a[k] + v * ab[k];
    return DOT3(q, q);
  }
  double d5 = DOT3(ab, cp), d6 = DOT3(ac, cp);
  if (d6 >= 0 && d5 <= d6)
    return DOT3(c, c);
  double vb = d5 * d2 - d1 * d6;
  if (vb <= 0 && d2 >= 0 && d6 <= 0)
  {
    double w = d2 / (d2 - d6);
    for (int k = 0; k < 3; k++) q[k] = a[k] + w * ac[k];
    return DOT3(q, q);
  }
  double va = d3 * d6 - d5 * d4;
  if (va <= 0 && (d4 - d3) >= 0 && (d5 - d6) >= 0)
  {
    double w = (d4 - d3) / ((d4 - d3) + (d5 - d6));
    for (int k = 0; k < 3; k++) q[k] = b[k] + w * (c[k] - b[k]);
    return DOT3(q, q);
  }
  double den = 1.0 / (va + vb + vc);
  double v = vb * den, w = vc * den;
  for (int k = 0; k < 3; k++) q[k] = a[k] + ab[k] * v + ac[k] * w;
  return DOT3(q, q);
#undef DOT3
}

/* Can the reference's interpolated normal (n0'(1-u-v) + n1' u) + n2' v of
 * this triangle (cpu/hit.c:38-40, nk' = the normalised vertex normals) be
 * exactly zero for some accepted (u, v)?  Only if 0 lies in (or within float
 * rounding of) the triangle the three unit normals span: each component is
 * a sum of three products of magnitude <= 1, rounded to a few 2^-24, and u,
 * v, 1-u-v may stray a few ulps outside [0, 1].  Distance < 1e-5 = "can". A
 * NaN normal (normalize of a zero vn) stays NaN, never zero. */
int rt_tri_normal_can_vanish(const float *nrm9)
{
  double n[3][3];
  for (int k = 0; k < 9; k++)
  {
    if (isnan(nrm9[k]))
      return 0;
    n[k / 3][k % 3] = nrm9[k];
  }
  return origin_tri_dist2(n[0], n[1], n[2]) < 1e-10;
}

int rt_flatten(const rt_scene *s, int accel, rt_flat_scene *out)
{
  memset(out, 0, sizeof *out);
  if (!s)
    return rt_set_error(RT_EINVAL, "null scene");
  size_t ntri = rt_scene_triangle_count(s);
  if (ntri >= 0x7fffffffu)
    return rt_set_error(RT_EINVAL, "too many triangles (%zu)", ntri);
  out->ntri = ntri;
  out->nobj = s->object_count;
  out->nlight = s->light_count;
  float *rec = malloc((ntri ? ntri : 1) * RT_TRI_FLOATS * sizeof(float));
  out->nrm = malloc((ntri ? ntri : 1) * 9 * sizeof(float));
  out->mat = calloc(s->object_count ? s->object_count : 1, RT_MAT_FLOATS * sizeof(float));
  out->light = calloc(s->light_count ? s->light_count : 1, RT_LIGHT_FLOATS * sizeof(float));
  float *pbox = malloc((ntri ? ntri : 1) * 6 * sizeof(float));
  if (!rec || !out->nrm || !out->mat || !out->light || !pbox)
  {
    free(rec);
    free(pbox);
    rt_flat_free(out);
    return rt_set_error(RT_ENOMEM, "flatten %zu triangles", ntri);
  }
  for (int a = 0; a < 3; a++)
  {
    out->scene_lo[a] = FLT_MAX;
    out->scene_hi[a] = -FLT_MAX;
  }
  size_t p = 0;
  for (size_t o = 0; o < s->object_count; o++)
  {
    const rt_object *ob = &s->objects[o];
    float *m = out->mat + RT_MAT_FLOATS * o;
    m[0] = ob->ka.x; m[1] = ob->ka.y; m[2] = ob->ka.z;
    m[3] = ob->kd.x; m[4] = ob->kd.y; m[5] = ob->kd.z;
    m[6] = ob->ks.x; m[7] = ob->ks.y; m[8] = ob->ks.z;
    m[9] = ob->ns;
    m[10] = ob->nr;
    m[11] = 0;
    for (unsigned t = 0; t < ob->triangle_count; t++, p++)
    {
      const rt_triangle *tr = &ob->triangles[t];
      rt_vec3 e1 = rt_v_sub(tr->vertex[1], tr->vertex[0]);
      rt_vec3 e2 = rt_v_sub(tr->vertex[2], tr->vertex[0]);
      float *r = rec + RT_TRI_FLOATS * p;
      r[0] = tr->vertex[0].x; r[1] = tr->vertex[0].y; r[2] = tr->vertex[0].z; r[3] = e1.x;
      r[4] = e1.y; r[5] = e1.z; r[6] = e2.x; r[7] = e2.y;
      r[8] = e2.z; r[9] = u2f((uint32_t)p); r[10] = u2f((uint32_t)o); r[11] = 0;
      float *nm = out->nrm + 9 * p;
      for (int k = 0; k < 3; k++)
      {
        rt_vec3 nn = rt_v_normalize(tr->normal[k]);
        nm[3 * k + 0] = nn.x;
        nm[3 * k + 1] = nn.y;
        nm[3 * k + 2] = nn.z;
      }
      float *pb = pbox + 6 * p;
      for (int a = 0; a < 3; a++)
      {
        float c0 = (&tr->vertex[0].x)[a], c1 = (&tr->vertex[1].x)[a], c2 = (&tr->vertex[2].x)[a];
        pb[a] = fminf(c0, fminf(c1, c2));
        pb[3 + a] = fmaxf(c0, fmaxf(c1, c2));
        if (pb[a] < out->scene_lo[a]) out->scene_lo[a] = pb[a];
        if (pb[3 + a] > out->scene_hi[a]) out->scene_hi[a] = pb[3 + a];
      }
    }
  }
  /* record flag RT_REC_ZERO_RISK on every triangle of an object that holds
   * a triangle whose interpolated normal can vanish (cpu/hit.c:79,99 skip
   * such an object when its closest triangle interpolates exactly zero) */
  for (size_t o = 0, p0 = 0; o < s->object_count; o++)
  {
    size_t n = s->objects[o].triangle_count;
    int risk = 0;
    for (size_t k = 0; k < n && !risk; k++)
      risk = rt_tri_normal_can_vanish(out->nrm + 9 * (p0 + k));
    if (risk)
      for (size_t k = 0; k < n; k++)
        rec[RT_TRI_FLOATS * (p0 + k) + 11] = u2f(RT_REC_ZERO_RISK_BIT);
    p0 += n;
  }
  for (size_t i = 0; i < s->light_count; i++)
  {
    const rt_light *l = &s->lights[i];
    float *L = out->light + RT_LIGHT_FLOATS * i;
    L[0] = u2f((uint32_t)l->type);
    L[1] = l->r; L[2] = l->g; L[3] = l->b;
    L[4] = l->v.x; L[5] = l->v.y; L[6] = l->v.z; L[7] = 0;
  }

  if (accel == RT_ACCEL_FLAT || ntri == 0)
  {
    out->tri = rec;
    out->nrec = ntri;
    free(pbox);
    return RT_OK;
  }
  if (accel != RT_ACCEL_OCTREE)
  {
    free(rec);
    free(pbox);
    rt_flat_free(out);
    return rt_set_error(RT_EINVAL, "unknown accel %d", accel);
  }

  /* root cell: the scene box made cubic (octants stay cubes) */
  dbox root;
  double ext = 0;
  for (int a = 0; a < 3; a++)
    ext = fmax(ext, (double)out->scene_hi[a] - out->scene_lo[a]);
  ext = ext * 1.0001 + 1e-6;
  for (int a = 0; a < 3; a++)
  {
    double c = 0.5 * ((double)out->scene_lo[a] + out->scene_hi[a]);
    root.lo[a] = c - 0.5 * ext;
    root.hi[a] = c + 0.5 * ext;
  }
  oct_input in = { rec, pbox, ext * 1e-6, RT_OCT_SIZE_STOP, RT_OCT_LEAF, RT_OCT_C_BOX,
                   RT_OCT_LEAF_CAP };
  const char *ev = getenv("RT_OCT_SIZE_STOP"); /* tuning knobs (tools/, not the API) */
  if (ev) in.size_stop = atof(ev);
  ev = getenv("RT_OCT_LEAF");
  if (ev) in.leaf_max = atoi(ev);
  ev = getenv("RT_OCT_C_BOX");
  if (ev) in.c_box = atof(ev);
  ev = getenv("RT_OCT_LEAF_CAP");
  if (ev) in.leaf_cap = atoi(ev);
  oct_tree b;
  if (build_octree(&in, ntri, &root, &b))
  {
    free(b.node);
    free(b.refs);
    free(rec);
    free(pbox);
    rt_flat_free(out);
    return rt_set_error(RT_ENOMEM, "octree build");
  }
  /* leaf-ordered triangle records (duplicated per leaf) */
  out->tri = malloc((b.nref ? b.nref : 1) * RT_TRI_FLOATS * sizeof(float));
  if (!out->tri)
  {
    free(b.node);
    free(b.refs);
    free(rec);
    free(pbox);
    rt_flat_free(out);
    return rt_set_error(RT_ENOMEM, "octree records");
  }
  for (size_t i = 0; i < b.nref; i++)
    memcpy(out->tri + RT_TRI_FLOATS * i, rec + RT_TRI_FLOATS * (size_t)b.refs[i],
           RT_TRI_FLOATS * sizeof(float));
  out->nrec = b.nref;
  out->node = b.node;
  out->nnode = b.nnode;
  out->root_count = 1;
  out->leaves = b.leaves;
  out->max_depth = b.max_depth;
  out->max_leaf = b.max_leaf;
  free(b.refs);
  free(rec);
  free(pbox);
  return RT_OK;
}

void rt_flat_free(rt_flat_scene *f)
{
  if (!f)
    return;
  free(f->tri);
  free(f->nrm);
  free(f->mat);
  free(f->light);
  free(f->node);
  memset(f, 0, sizeof *f);
}

/* ------------------------------------------------------- host-only checks */

int rt_accel_build_info(const rt_scene *s, int accel, rt_accel_info *info)
{
  if (!s || !info)
    return rt_set_error(RT_EINVAL, "null argument");
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  rt_flat_scene f;
  int rc = rt_flatten(s, accel, &f);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  if (rc)
    return rc;
  memset(info, 0, sizeof *info);
  info->triangles = f.ntri;
  info->tri_refs = f.nrec;
  info->nodes = f.nnode;
  info->leaves = f.leaves;
  info->max_depth = f.max_depth;
  info->max_leaf = f.max_leaf;
  info->tri_record_bytes = RT_TRI_FLOATS * sizeof(float);
  info->node_record_bytes = RT_NODE_FLOATS * sizeof(float);
  info->device_bytes = (f.nrec * RT_TRI_FLOATS + f.ntri * 9 + f.nobj * RT_MAT_FLOATS +
                        f.nlight * RT_LIGHT_FLOATS + f.nnode * RT_NODE_FLOATS) * sizeof(float);
  info->build_seconds = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
  rt_flat_free(&f);
  return RT_OK;
}

static int box_contains(const float *outer, const float *lo, const float *hi)
{
  for (int a = 0; a < 3; a++)
    if (lo[a] < outer[a] || hi[a] > outer[4 + a])
      return 0;
  return 1;
}

int rt_accel_validate(const rt_scene *s, int accel)
{
  rt_flat_scene f;
  int rc = rt_flatten(s, accel, &f);
  if (rc)
    return rc;
  rc = rt_flat_validate(&f);
  rt_flat_free(&f);
  return rc;
}

/* index of a record of prim `prim` in leaf `n` (it holds one) */
static size_t leaf_rec_of(const rt_flat_scene *f, uint32_t n, uint32_t prim)
{
  const float *nd = f->node + RT_NODE_FLOATS * (size_t)n;
  uint32_t first, info;
  memcpy(&first, &nd[3], 4);
  memcpy(&info, &nd[7], 4);
  for (uint32_t k = 0; k < RT_LEAF_COUNT(info); k++)
  {
    uint32_t q;
    memcpy(&q, &f->tri[RT_TRI_FLOATS * (size_t)(first + k) + 9], 4);
    if (q == prim)
      return first + k;
  }
  return first;
}

/* Coverage: every point of a triangle must lie in the box of some leaf that
 * holds it -- otherwise a ray through that point could skip the triangle (a
 * cell wrongly dropped by a builder's plane test or clipping would pass the
 * per-leaf overlap checks).  Checked on a barycentric grid of 28 points per
 * triangle (vertices, edges, interior), each against the prim's own leaves,
 * with the builders' rounding slack. */
static int validate_coverage(const rt_flat_scene *f, float scene_ext)
{
  size_t *cnt = calloc(f->ntri + 1, sizeof *cnt);
  uint32_t *leaf_of = malloc((f->nrec ? f->nrec : 1) * sizeof *leaf_of);
  if (!cnt || !leaf_of)
  {
    free(cnt);
    free(leaf_of);
    return rt_set_error(RT_ENOMEM, "validate coverage");
  }
  /* CSR prim -> leaves holding a record of it */
  for (int pass = 0; pass < 2; pass++)
  {
    for (size_t n = 0; n < f->nnode; n++)
    {
      const float *nd = f->node + RT_NODE_FLOATS * n;
      uint32_t first, info;
      memcpy(&first, &nd[3], 4);
      memcpy(&info, &nd[7], 4);
      if (!(info & RT_NODE_LEAF))
        continue;
      for (uint32_t k = 0; k < RT_LEAF_COUNT(info); k++)
      {
        uint32_t prim;
        memcpy(&prim, &f->tri[RT_TRI_FLOATS * (size_t)(first + k) + 9], 4);
        if (pass == 0)
          cnt[prim + 1]++;
        else
          leaf_of[cnt[prim]++] = (uint32_t)n;
      }
    }
    if (pass == 0)
      for (size_t p = 0; p < f->ntri; p++)
        cnt[p + 1] += cnt[p];
    else
      for (size_t p = f->ntri; p > 0; p--) /* the fill advanced cnt[p] to the next prim's start */
        cnt[p] = cnt[p - 1];
    if (pass == 1)
      cnt[0] = 0;
  }
  int rc = RT_OK;
  const int N = 6;
  for (size_t p = 0; p < f->ntri && !rc; p++)
  {
    /* the prim-order record: a leaf record of prim p carries the same floats */
    const float *r = f->tri + RT_TRI_FLOATS * (size_t)leaf_rec_of(f, leaf_of[cnt[p]], (uint32_t)p);
    for (int i = 0; i <= N && !rc; i++)
      for (int j = 0; i + j <= N && !rc; j++)
      {
        double u = (double)i / N, v = (double)j / N, x[3];
        for (int a = 0; a < 3; a++)
          x[a] = (double)r[a] + u * (double)r[3 + a] + v * (double)r[6 + a];
        int in = 0;
        for (size_t q = cnt[p]; q < cnt[p + 1] && !in; q++)
        {
          const float *nd = f->node + RT_NODE_FLOATS * (size_t)leaf_of[q];
          in = 1;
          for (int a = 0; a < 3 && in; a++)
          {
            double sl = 1e-5 * fabs(x[a]) + 2e-6 * scene_ext + 1e-6;
            in = x[a] >= (double)nd[a] - sl && x[a] <= (double)nd[4 + a] + sl;
          }
        }
        if (!in)
          rc = rt_set_error(RT_EINVAL, "prim %zu: point (%g, %g, %g) of the triangle lies in none "
                            "of its %zu leaves' boxes", p, x[0], x[1], x[2], cnt[p + 1] - cnt[p]);
      }
  }
  free(cnt);
  free(leaf_of);
  return rc;
}

/* Invariants of a flattened scene image (host-built, or downloaded from a
 * device build by rt_hip_accel_validate). */
int rt_flat_validate(const rt_flat_scene *fp)
{
  const rt_flat_scene f = *fp;
  int rc = RT_OK;
  if (!f.nnode)
    return f.nrec == f.ntri ? RT_OK : rt_set_error(RT_EINVAL, "flat: %zu records for %zu prims",
                                                   f.nrec, f.ntri);
  float scene_ext = 0;
  for (int a = 0; a < 3; a++)
    scene_ext = fmaxf(scene_ext, f.scene_hi[a] - f.scene_lo[a]);
  unsigned char *seen = calloc(f.ntri ? f.ntri : 1, 1);
  if (!seen)
    return rt_set_error(RT_ENOMEM, "validate");
  for (size_t n = 0; n < f.nnode && !rc; n++)
  {
    const float *nd = f.node + RT_NODE_FLOATS * n;
    uint32_t first, cnt;
    memcpy(&first, &nd[3], 4);
    memcpy(&cnt, &nd[7], 4);
    if (cnt & RT_NODE_LEAF)
    {
      cnt = RT_LEAF_COUNT(cnt);
      if ((size_t)first + cnt > f.nrec)
        rc = rt_set_error(RT_EINVAL, "leaf %zu: records out of range", n);
      for (uint32_t k = 0; k < cnt && !rc; k++)
      {
        const float *r = f.tri + RT_TRI_FLOATS * (size_t)(first + k);
        uint32_t prim;
        memcpy(&prim, &r[9], 4);
        if (prim >= f.ntri)
        {
          rc = rt_set_error(RT_EINVAL, "leaf %zu: prim %u out of range", n, prim);
          break;
        }
        seen[prim] = 1;
        /* exact float vertices: v0, v0+e1 and v0+e2 may round, so rebuild the
         * box from the record the same way the builder's bbox saw them */
        float lo[3], hi[3];
        for (int a = 0; a < 3; a++)
        {
          float v0 = r[a], e1 = r[3 + a], e2 = r[6 + a];
          float c1 = v0 + e1, c2 = v0 + e2;
          lo[a] = fminf(v0, fminf(c1, c2));
          hi[a] = fmaxf(v0, fmaxf(c1, c2));
          /* the builder inserts triangles that touch a cell within its pad
           * (2e-6 of the scene extent here), while the box is clipped to the cell */
          float slack = 1e-5f * (fabsf(lo[a]) + fabsf(hi[a])) + 2e-6f * scene_ext + 1e-6f;
          lo[a] -= slack;
          hi[a] += slack;
        }
        /* boxes are clipped to their cell: the triangle must overlap it */
        for (int a = 0; a < 3 && !rc; a++)
          if (hi[a] < nd[a] || lo[a] > nd[4 + a])
            rc = rt_set_error(RT_EINVAL, "leaf %zu box misses prim %u (axis %d: tri [%g,%g] box [%g,%g])", n, prim, a, lo[a], hi[a], nd[a], nd[4 + a]);
      }
    }
    else
    {
      uint32_t mask = RT_NODE_MASK(cnt);
      cnt = RT_NODE_COUNT(cnt);
      if (cnt == 0 || cnt > 8 || (uint32_t)__builtin_popcount(mask) != cnt ||
          (size_t)first + cnt > f.nnode || first <= n)
        rc = rt_set_error(RT_EINVAL, "node %zu: bad children [%u,+%u) mask %#x", n, first, cnt,
                          mask);
      for (uint32_t c = 0; c < cnt && !rc; c++)
      {
        const float *ch = f.node + RT_NODE_FLOATS * (size_t)(first + c);
        if (!box_contains(nd, ch, ch + 4))
          rc = rt_set_error(RT_EINVAL, "node %zu box misses child %u", n, first + c);
      }
    }
  }
  for (size_t p = 0; p < f.ntri && !rc; p++)
    if (!seen[p])
      rc = rt_set_error(RT_EINVAL, "prim %zu in no leaf", p);
  free(seen);
  if (!rc)
    rc = validate_coverage(&f, scene_ext);
  return rc;
}
