/* TEST INFRASTRUCTURE — CPU oracle (see crt_oracle.h). Never linked into the product.
 *
 * Plain-C restatement of the reference's render path, each function following the reference
 * line by line in operation order (compiled with -ffp-contract=off like the reference's ISO
 * C++20 x86-64 build). Radiance is accumulated exactly as the reference's recursion does
 * (camera.h:233-234), so for the same per-sample RNG stream this oracle reproduces the
 * reference's per-pixel output bit for bit (tests/test_oracle.py).
 * Reference paths are relative to DeltaPavonis/cpp_raytracer.
 */
#include "crt_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ---- Vec3D (math/vec3d.h) --------------------------------------------------------------- */
typedef struct { double x, y, z; } V3;
static inline V3 mk(double x, double y, double z) { V3 r = {x, y, z}; return r; }
static inline V3 add(V3 a, V3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }     /* :98  */
static inline V3 sub(V3 a, V3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }     /* :100 */
static inline V3 mul(V3 a, double d) { return mk(a.x * d, a.y * d, a.z * d); }       /* :102 */
static inline V3 divd(V3 a, double d) { return mul(a, 1 / d); }                      /* :34  */
static inline V3 neg(V3 a) { return mk(-a.x, -a.y, -a.z); }                          /* :25  */
static inline double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }   /* :114 */
static inline V3 cross(V3 a, V3 b) {                                                 /* :116 */
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline double mag2(V3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }        /* :39  */
static inline double mag(V3 a) { return sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }  /* :37  */
static inline V3 unit(V3 a) { return divd(a, mag(a)); }                             /* :127 */
static inline V3 ld(const double* p) { return mk(p[0], p[1], p[2]); }
static inline double comp(V3 v, int k) { return k == 0 ? v.x : (k == 1 ? v.y : v.z); }

/* ---- RNG (util/rand_util.h:85-117) with per-sample state -------------------------------- */
uint32_t oracle_sample_seed(uint32_t base, uint32_t pixel, uint32_t sample) {
    uint64_t z = ((uint64_t)pixel << 32) | sample;
    z += (uint64_t)base * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (uint32_t)(z ^ (z >> 32));
}
static inline double rnd(uint32_t* s, double lo, double hi) {
    *s = 1664525u * *s + 1013904223u;
    const double scale = 1 / (double)(UINT32_MAX - 1);
    return lo + (hi - lo) * (double)*s * scale;
}
static V3 random_unit_vector(uint32_t* s) { /* vec3d.h:64-75 */
    V3 r;
    do {
        double x = rnd(s, -1, 1), y = rnd(s, -1, 1), z = rnd(s, -1, 1); /* braced: x, y, z */
        r = mk(x, y, z);
    } while (!(mag2(r) < 1));
    return unit(r);
}

/* ---- std::midpoint<double> of libstdc++ (interval.h:31) --------------------------------- */
static double midpoint(double a, double b) {
    const double lo = DBL_MIN * 2, hi = DBL_MAX / 2;
    const double aa = a < 0 ? -a : a, ab = b < 0 ? -b : b;
    if (aa <= hi && ab <= hi) return (a + b) / 2;
    if (aa < lo) return a + b / 2;
    if (ab < lo) return a / 2 + b;
    return a / 2 + b / 2;
}

/* ---- AABB (acceleration/aabb.h) as 6 doubles: x.min x.max y.min y.max z.min z.max -------- */
static void box_empty(double* b) {
    for (int k = 0; k < 3; ++k) { b[2 * k] = INFINITY; b[2 * k + 1] = -INFINITY; }
}
static void box_merge(double* b, const double* o) { /* aabb.h:177-183, interval.h:49-52 */
    for (int k = 0; k < 6; k += 2) { b[k] = fmin(b[k], o[k]); b[k + 1] = fmax(b[k + 1], o[k + 1]); }
}
static void box_merge_pt(double* b, V3 p) { /* aabb.h:186-191 */
    for (int k = 0; k < 3; ++k) {
        b[2 * k] = fmin(b[2 * k], comp(p, k));
        b[2 * k + 1] = fmax(b[2 * k + 1], comp(p, k));
    }
}
static double box_area(const double* b) { /* aabb.h:29-31 */
    double sx = b[1] - b[0], sy = b[3] - b[2], sz = b[5] - b[4];
    return 2 * (sx * sx + sy * sy + sz * sz);
}
static V3 box_centroid(const double* b) { /* aabb.h:27 */
    return mk(midpoint(b[0], b[1]), midpoint(b[2], b[3]), midpoint(b[4], b[5]));
}

/* ---- primitives --------------------------------------------------------------------------- */
typedef struct {
    int kind; /* CRT_SPHERE / CRT_PARALLELOGRAM */
    uint32_t mat;
    V3 c; double r;           /* sphere.h:16-18 */
    V3 v, s1, s2, n, sn;      /* parallelogram.h:138-170 */
    double box[6];
} Prim;

static Prim make_sphere(V3 c, double r, uint32_t mat) { /* sphere.h:112-122 */
    Prim p;
    memset(&p, 0, sizeof p);
    p.kind = CRT_SPHERE; p.mat = mat; p.c = c; p.r = r;
    V3 rv = mk(r, r, r);
    box_empty(p.box);
    box_merge_pt(p.box, sub(c, rv));
    box_merge_pt(p.box, add(c, rv));
    return p;
}
static Prim make_quad(V3 v, V3 s1, V3 s2, uint32_t mat) { /* parallelogram.h:269-296 */
    Prim p;
    memset(&p, 0, sizeof p);
    p.kind = CRT_PARALLELOGRAM; p.mat = mat; p.v = v; p.s1 = s1; p.s2 = s2;
    V3 n = cross(s1, s2);
    p.n = unit(n);
    p.sn = divd(n, mag2(n));
    box_empty(p.box);
    box_merge_pt(p.box, v);
    box_merge_pt(p.box, add(v, s1));
    box_merge_pt(p.box, add(v, s2));
    box_merge_pt(p.box, add(add(v, s1), s2));
    for (int k = 0; k < 3; ++k) { /* ensure_min_axis_length(1e-4), aabb.h:197-202 */
        double sz = p.box[2 * k + 1] - p.box[2 * k];
        if (sz < 1e-4) {
            double pad = (1e-4 - (p.box[2 * k + 1] - p.box[2 * k])) / 2;
            p.box[2 * k] -= pad;
            p.box[2 * k + 1] += pad;
        }
    }
    return p;
}

/* Scene::get_primitive_components (scene.h:85-106); Box -> six faces (box.h:53-84) */
static Prim* flatten(const crt_object* objs, size_t no, size_t* np) {
    size_t n = 0;
    for (size_t i = 0; i < no; ++i) n += objs[i].kind == CRT_BOX ? 6 : 1;
    Prim* p = (Prim*)malloc(sizeof(Prim) * (n ? n : 1));
    size_t k = 0;
    for (size_t i = 0; i < no; ++i) {
        const crt_object* o = &objs[i];
        if (o->kind == CRT_SPHERE) {
            p[k++] = make_sphere(ld(o->v), o->v[3], o->material);
        } else if (o->kind == CRT_PARALLELOGRAM) {
            p[k++] = make_quad(ld(o->v), ld(o->v + 3), ld(o->v + 6), o->material);
        } else {
            double a[3], b[3];
            for (int j = 0; j < 3; ++j) { a[j] = fmin(o->v[j], o->v[3 + j]); b[j] = fmax(o->v[j], o->v[3 + j]); }
            V3 mn = ld(a), mx = ld(b);
            V3 sx = mk(mx.x - mn.x, 0, 0), sy = mk(0, mx.y - mn.y, 0), sz = mk(0, 0, mx.z - mn.z);
            p[k++] = make_quad(mn, sx, sy, o->material);
            p[k++] = make_quad(mn, sx, sz, o->material);
            p[k++] = make_quad(mn, sy, sz, o->material);
            p[k++] = make_quad(mx, neg(sx), neg(sy), o->material);
            p[k++] = make_quad(mx, neg(sx), neg(sz), o->material);
            p[k++] = make_quad(mx, neg(sy), neg(sz), o->material);
        }
    }
    *np = n;
    return p;
}

/* ---- BVH build (bvh.h:183-461) and preorder flattening (bvh.h:468-550) -------------------- */
typedef struct TNode {
    double box[6];
    struct TNode *l, *r;
    size_t first, count;
    uint32_t axis;
} TNode;

typedef struct {
    const Prim* prims;
    uint32_t* order;
    size_t nb, max_leaf, total;
} Build;

static size_t bucket_of(const Build* B, uint32_t prim, int axis, const double* cb) {
    V3 c = box_centroid(B->prims[prim].box);
    double offset = (comp(c, axis) - cb[2 * axis]) / (cb[2 * axis + 1] - cb[2 * axis]);
    size_t b = (size_t)((double)B->nb * offset);
    if (b == B->nb) --b;
    return b;
}

/* libstdc++'s std::partition for bidirectional iterators (bvh.h:417 calls std::partition) */
static size_t partition(const Build* B, size_t first, size_t last, int axis, const double* cb,
                        size_t best) {
    uint32_t* a = B->order;
    for (;;) {
        for (;;) {
            if (first == last) return first;
            if (bucket_of(B, a[first], axis, cb) <= best) ++first;
            else break;
        }
        --last;
        for (;;) {
            if (first == last) return first;
            if (!(bucket_of(B, a[last], axis, cb) <= best)) --last;
            else break;
        }
        uint32_t t = a[first]; a[first] = a[last]; a[last] = t;
        ++first;
    }
}

static TNode* build(Build* B, size_t lo, size_t hi) {
    TNode* n = (TNode*)calloc(1, sizeof(TNode));
    ++B->total;
    box_empty(n->box);
    for (size_t i = lo; i < hi; ++i) box_merge(n->box, B->prims[B->order[i]].box);
    if (hi - lo == 1) { n->first = lo; n->count = 1; return n; }
    double cb[6];
    box_empty(cb);
    for (size_t i = lo; i < hi; ++i) box_merge_pt(cb, box_centroid(B->prims[B->order[i]].box));
    double min_cost = INFINITY;
    int best_axis = 0;
    size_t best_bucket = 0;
    size_t* bn = (size_t*)malloc(sizeof(size_t) * B->nb);
    double* bb = (double*)malloc(sizeof(double) * 6 * B->nb);
    double* costs = (double*)malloc(sizeof(double) * B->nb);
    for (int axis = 0; axis < 3; ++axis) {
        if (cb[2 * axis + 1] - cb[2 * axis] <= 0) continue; /* is_empty_exclusive, bvh.h:244 */
        for (size_t k = 0; k < B->nb; ++k) { bn[k] = 0; box_empty(bb + 6 * k); }
        for (size_t i = lo; i < hi; ++i) {
            size_t b = bucket_of(B, B->order[i], axis, cb);
            bn[b]++;
            box_merge(bb + 6 * b, B->prims[B->order[i]].box);
        }
        double before[6];
        box_empty(before);
        size_t nbef = 0;
        for (size_t k = 0; k + 1 < B->nb; ++k) { /* bvh.h:348-356 */
            box_merge(before, bb + 6 * k);
            nbef += bn[k];
            costs[k] = box_area(before) * (double)nbef;
        }
        double after[6];
        box_empty(after);
        size_t naft = 0;
        for (long k = (long)B->nb - 2; k >= 0; --k) { /* bvh.h:360-369 (bucket k itself) */
            box_merge(after, bb + 6 * k);
            naft += bn[k];
            costs[k] += box_area(after) * (double)naft;
        }
        for (size_t k = 0; k + 1 < B->nb; ++k) {
            if (costs[k] < min_cost) { min_cost = costs[k]; best_axis = axis; best_bucket = k; }
        }
    }
    free(bn); free(bb); free(costs);
    if (isinf(min_cost)) { n->first = lo; n->count = hi - lo; return n; } /* bvh.h:395-397 */
    double leaf_cost = (double)(hi - lo);
    if (hi - lo > B->max_leaf || min_cost < leaf_cost) {
        size_t mid = partition(B, lo, hi, best_axis, cb, best_bucket);
        n->l = build(B, lo, mid);
        n->r = build(B, mid, hi);
        n->axis = (uint32_t)best_axis;
        return n;
    }
    n->first = lo;
    n->count = hi - lo;
    return n;
}

static void flatten_tree(TNode* t, crt_bvh_node* out, size_t* next) {
    size_t me = (*next)++;
    crt_bvh_node n;
    memset(&n, 0, sizeof n);
    memcpy(n.bounds, t->box, sizeof n.bounds);
    if (!t->l) {
        n.index = (uint32_t)t->first;
        n.count = (uint32_t)t->count;
        out[me] = n;
    } else {
        flatten_tree(t->l, out, next);
        n.index = (uint32_t)*next;
        n.axis = t->axis;
        out[me] = n;
        flatten_tree(t->r, out, next);
    }
}

static void free_tree(TNode* t) {
    if (!t) return;
    free_tree(t->l);
    free_tree(t->r);
    free(t);
}

typedef struct {
    Prim* prims;          /* in slot (BVH) order */
    uint32_t* order;      /* slot -> primitive index */
    size_t np;
    crt_bvh_node* nodes;
    size_t nn;
    size_t depth;
    const crt_material* mats;
} World;

static size_t tree_depth(const crt_bvh_node* nodes, size_t i) {
    if (nodes[i].count > 0) return 1;
    size_t l = tree_depth(nodes, i + 1), r = tree_depth(nodes, nodes[i].index);
    return 1 + (l > r ? l : r);
}

static int world_make(const crt_material* mats, const crt_object* objs, size_t no, uint32_t nb,
                      uint32_t max_leaf, World* w) {
    memset(w, 0, sizeof *w);
    w->mats = mats;
    Prim* p = flatten(objs, no, &w->np);
    w->order = (uint32_t*)malloc(sizeof(uint32_t) * (w->np ? w->np : 1));
    for (size_t i = 0; i < w->np; ++i) w->order[i] = (uint32_t)i;
    if (w->np == 0) {
        w->nodes = (crt_bvh_node*)calloc(1, sizeof(crt_bvh_node));
        for (int k = 0; k < 3; ++k) { w->nodes[0].bounds[2 * k] = INFINITY; w->nodes[0].bounds[2 * k + 1] = -INFINITY; }
        w->nn = 1;
        w->prims = p;
        w->depth = 1;
        return 0;
    }
    Build B = {p, w->order, nb, max_leaf, 0};
    TNode* root = build(&B, 0, w->np);
    w->nodes = (crt_bvh_node*)calloc(B.total, sizeof(crt_bvh_node));
    size_t next = 0;
    flatten_tree(root, w->nodes, &next);
    free_tree(root);
    w->nn = B.total;
    /* primitives in slot order (the BVH's permuted copy, bvh.h:164) */
    w->prims = (Prim*)malloc(sizeof(Prim) * w->np);
    for (size_t i = 0; i < w->np; ++i) w->prims[i] = p[w->order[i]];
    free(p);
    w->depth = tree_depth(w->nodes, 0);
    return 0;
}

static void world_free(World* w) {
    free(w->prims);
    free(w->order);
    free(w->nodes);
}

/* ---- hit tests ---------------------------------------------------------------------------- */
typedef struct {
    double t;
    V3 p, n;        /* hit point, normal facing the ray (hittable.h:46-71) */
    int front;
    uint32_t mat;
    size_t slot;
} Hit;

static int hit_sphere(const Prim* s, V3 o, V3 d, double tmin, double tmax, double* t) { /* sphere.h:45-96 */
    V3 oc = sub(o, s->c);
    double a = dot(d, d);
    double b = dot(d, oc);
    double c = dot(oc, oc) - s->r * s->r;
    double disc = b * b - a * c;
    if (disc < 0) return 0;
    double sq = sqrt(disc);
    double root = (-b - sq) / a;
    if (!(tmin < root && root < tmax)) {
        root = (-b + sq) / a;
        if (!(tmin < root && root < tmax)) return 0;
    }
    *t = root;
    return 1;
}

static int hit_quad(const Prim* q, V3 o, V3 d, double tmin, double tmax, double* t) { /* parallelogram.h:177-240 */
    double den = dot(q->n, d);
    if (fabs(den) < 1e-9) return 0;
    double ht = dot(q->n, sub(q->v, o)) / den;
    if (!(tmin < ht && ht < tmax)) return 0;
    V3 p = add(o, mul(d, ht));
    V3 w = sub(p, q->v);
    double alpha = dot(q->sn, cross(w, q->s2));
    double beta = dot(q->sn, cross(q->s1, w));
    if (0 <= alpha && alpha <= 1 && 0 <= beta && beta <= 1) { *t = ht; return 1; }
    return 0;
}

static int aabb_hit(const double* b, V3 o, V3 inv, const int* ng, double tmin, double tmax) { /* aabb.h:132-174 */
    double x_tmin = (b[0 + ng[0]] - o.x) * inv.x;
    double x_tmax = (b[1 - ng[0]] - o.x) * inv.x;
    double y_tmin = (b[2 + ng[1]] - o.y) * inv.y;
    double y_tmax = (b[3 - ng[1]] - o.y) * inv.y;
    if (x_tmin > y_tmax || y_tmin > x_tmax) return 0;
    if (y_tmin > x_tmin) x_tmin = y_tmin;
    if (y_tmax < x_tmax) x_tmax = y_tmax;
    double z_tmin = (b[4 + ng[2]] - o.z) * inv.z;
    double z_tmax = (b[5 - ng[2]] - o.z) * inv.z;
    if (x_tmin > z_tmax || z_tmin > x_tmax) return 0;
    if (z_tmin > x_tmin) x_tmin = z_tmin;
    if (z_tmax < x_tmax) x_tmax = z_tmax;
    return (x_tmin < tmax) && (x_tmax > tmin);
}

/* BVH::hit_by (bvh.h:585-715) */
static int bvh_hit(const World* w, V3 o, V3 d, double tmin, double tmax, Hit* h, oracle_stats* st,
                   size_t* stack) {
    int found = 0;
    size_t sp = 0, cur = 0;
    V3 inv = mk(1 / d.x, 1 / d.y, 1 / d.z);
    int ng[3] = {d.x < 0, d.y < 0, d.z < 0};
    double t;
    for (;;) {
        const crt_bvh_node* n = &w->nodes[cur];
        if (st) st->nodes_visited++;
        if (aabb_hit(n->bounds, o, inv, ng, tmin, tmax)) {
            if (n->count > 0) {
                for (size_t i = n->index; i < (size_t)n->index + n->count; ++i) {
                    const Prim* p = &w->prims[i];
                    int hit;
                    if (p->kind == CRT_SPHERE) { if (st) st->sphere_tests++; hit = hit_sphere(p, o, d, tmin, tmax, &t); }
                    else { if (st) st->parallelogram_tests++; hit = hit_quad(p, o, d, tmin, tmax, &t); }
                    if (hit) { tmax = t; h->slot = i; found = 1; }
                }
                if (sp == 0) break;
                cur = stack[--sp];
            } else if (ng[n->axis]) {
                stack[sp++] = cur + 1;
                cur = n->index;
            } else {
                stack[sp++] = n->index;
                cur = cur + 1;
            }
        } else {
            if (sp == 0) break;
            cur = stack[--sp];
        }
    }
    if (found) { /* hit_info of the closest primitive (hittable.h:46-71) */
        const Prim* p = &w->prims[h->slot];
        h->t = tmax;
        h->p = add(o, mul(d, tmax));
        V3 out = p->kind == CRT_SPHERE ? divd(sub(h->p, p->c), p->r) : p->n;
        if (dot(d, out) > 0) { h->n = neg(out); h->front = 0; }
        else { h->n = out; h->front = 1; }
        h->mat = p->mat;
    }
    return found;
}

/* ---- materials (base/material.h) ------------------------------------------------------------ */
static V3 reflected(V3 dir, V3 n) { return sub(dir, mul(n, 2 * dot(dir, n))); } /* vec3d.h:144-155 */

/* returns 1 and sets (nd, att) when scattered */
static int scatter(const crt_material* m, V3 d, const Hit* h, uint32_t* rng, V3* nd, double att[3]) {
    switch (m->kind) {
        case CRT_LAMBERTIAN: { /* material.h:64-86 */
            V3 sd = add(h->n, random_unit_vector(rng));
            if (fabs(sd.x) < 1e-8 && fabs(sd.y) < 1e-8 && fabs(sd.z) < 1e-8) sd = h->n;
            *nd = sd;
            att[0] = m->color[0]; att[1] = m->color[1]; att[2] = m->color[2];
            return 1;
        }
        case CRT_METAL: { /* material.h:116-139 */
            V3 r = reflected(unit(d), h->n);
            V3 sd = add(r, mul(random_unit_vector(rng), m->param));
            if (dot(h->n, sd) < 0) return 0;
            *nd = sd;
            att[0] = m->color[0]; att[1] = m->color[1]; att[2] = m->color[2];
            return 1;
        }
        case CRT_DIELECTRIC: { /* material.h:185-218, vec3d.h:168-200, material.h:175-181 */
            double ratio = h->front ? 1. / m->param : m->param / 1.;
            V3 u = unit(d);
            double cos_t = fmin(dot(neg(u), h->n), 1.);
            double sin_t = sqrt(1 - cos_t * cos_t);
            V3 dir;
            if (ratio * sin_t > 1) {
                dir = reflected(u, h->n);
            } else {
                V3 perp = mul(add(u, mul(h->n, cos_t)), ratio);
                V3 para = mul(h->n, -sqrt(fabs(1 - mag2(perp))));
                dir = add(perp, para);
                double c2 = fmin(dot(neg(u), h->n), 1.);
                double r0 = (1 - ratio) / (1 + ratio);
                r0 *= r0;
                if (rnd(rng, 0, 1) < r0 + (1 - r0) * pow(1 - c2, 5)) dir = reflected(u, h->n);
            }
            *nd = dir;
            att[0] = att[1] = att[2] = 1;
            return 1;
        }
        default: /* DiffuseLight: never scatters (material.h:248-256) */
            return 0;
    }
}

/* Camera::ray_color (camera.h:205-258), recursive exactly like the reference */
static void ray_color(const World* w, const crt_camera* cam, V3 o, V3 d, uint32_t depth,
                      uint32_t* rng, double out[3], oracle_stats* st, size_t* stack) {
    if (depth == 0) { out[0] = out[1] = out[2] = 0; return; }
    if (st) st->rays++;
    Hit h;
    if (bvh_hit(w, o, d, cam->t_min, INFINITY, &h, st, stack)) {
        const crt_material* m = &w->mats[h.mat];
        double e[3] = {0, 0, 0};
        if (m->kind == CRT_DIFFUSE_LIGHT) { /* emit(): intensity * colour (material.h:261-263) */
            e[0] = m->color[0] * m->param; e[1] = m->color[1] * m->param; e[2] = m->color[2] * m->param;
        }
        V3 nd;
        double att[3];
        if (scatter(m, d, &h, rng, &nd, att)) {
            double next[3];
            ray_color(w, cam, h.p, nd, depth - 1, rng, next, st, stack);
            out[0] = e[0] + att[0] * next[0];
            out[1] = e[1] + att[1] * next[1];
            out[2] = e[2] + att[2] * next[2];
        } else {
            out[0] = e[0]; out[1] = e[1]; out[2] = e[2];
        }
    } else {
        out[0] = cam->background[0]; out[1] = cam->background[1]; out[2] = cam->background[2];
    }
}

/* ---- Camera::init (camera.h:87-157) ----------------------------------------------------- */
int oracle_camera(const crt_camera_settings* s, crt_camera* c) {
    if (!s || !c || s->image_w == 0 || s->image_h == 0) return -1;
    memset(c, 0, sizeof *c);
    c->image_w = s->image_w; c->image_h = s->image_h;
    c->samples_per_pixel = s->samples_per_pixel; c->max_depth = s->max_depth;
    double aspect = (double)s->image_w / (double)s->image_h;
    V3 center = ld(s->center);
    V3 dir = s->has_lookat ? sub(ld(s->lookat), center) : ld(s->direction);
    double focal = s->has_focus_dist ? s->focus_dist : mag(dir);
    double vw, vh;
    if (s->fov_is_vertical) { vh = 2 * focal * tan(s->fov / 2); vw = vh * aspect; }
    else { vw = 2 * focal * tan(s->fov / 2); vh = vw / aspect; }
    V3 bz = neg(unit(dir));
    V3 bx = unit(cross(ld(s->up), bz));
    V3 by = cross(bz, bx);
    V3 xv = mul(bx, vw), yv = mul(by, -vh);
    V3 pdx = divd(xv, (double)s->image_w), pdy = divd(yv, (double)s->image_h);
    V3 ulc = sub(sub(sub(center, mul(bz, focal)), divd(xv, 2)), divd(yv, 2));
    V3 p00 = add(add(ulc, divd(pdx, 2)), divd(pdy, 2));
    double rad = focal * tan(s->defocus_angle / 2);
    V3 ddx = mul(bx, rad), ddy = mul(by, rad);
    double* dst[] = {c->origin, c->pixel00, c->pixel_delta_x, c->pixel_delta_y, c->defocus_disk_x, c->defocus_disk_y};
    V3 src[] = {center, p00, pdx, pdy, ddx, ddy};
    for (int i = 0; i < 6; ++i) { dst[i][0] = src[i].x; dst[i][1] = src[i].y; dst[i][2] = src[i].z; }
    c->defocus_angle = s->defocus_angle;
    for (int k = 0; k < 3; ++k) c->background[k] = s->background[k];
    c->t_min = 0.00001;
    return 0;
}

/* Camera::random_ray_through_pixel (camera.h:184-200; g++ draws the pixel_delta_y jitter first) */
static void primary_ray(const crt_camera* c, size_t row, size_t col, uint32_t* rng, V3* o, V3* d) {
    V3 origin = ld(c->origin);
    if (!(c->defocus_angle <= 0)) { /* random_point_in_defocus_disk, camera.h:160-168 */
        double vx, vy;
        do {
            vx = rnd(rng, -1, 1);
            vy = rnd(rng, -1, 1);
        } while (!(vx * vx + vy * vy + 0 * 0 < 1));
        origin = add(add(ld(c->origin), mul(ld(c->defocus_disk_x), vx)), mul(ld(c->defocus_disk_y), vy));
    }
    V3 center = add(add(ld(c->pixel00), mul(ld(c->pixel_delta_y), (double)row)), mul(ld(c->pixel_delta_x), (double)col));
    double uy = rnd(rng, -0.5, 0.5);
    double ux = rnd(rng, -0.5, 0.5);
    V3 sample = add(add(center, mul(ld(c->pixel_delta_x), ux)), mul(ld(c->pixel_delta_y), uy));
    *o = origin;
    *d = sub(sample, origin);
}

int oracle_render(const crt_material* mats, size_t nm, const crt_object* objs, size_t no,
                  const crt_camera_settings* s, uint32_t base_seed, int threads, uint32_t r0,
                  uint32_t r1, uint32_t c0, uint32_t c1, double* rgb, double* samples,
                  oracle_stats* stats) {
    (void)nm;
    crt_camera cam;
    if (oracle_camera(s, &cam)) return -1;
    World w;
    world_make(mats, objs, no, 32, 12, &w);
    const size_t W = c1 - c0, spp = cam.samples_per_pixel;
    oracle_stats total;
    memset(&total, 0, sizeof total);
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#else
    (void)threads;
#endif
#pragma omp parallel
    {
        oracle_stats mine;
        memset(&mine, 0, sizeof mine);
        size_t* stack = (size_t*)malloc(sizeof(size_t) * (w.depth + 2));
#pragma omp for schedule(dynamic)
        for (long row = (long)r0; row < (long)r1; ++row) {
            for (size_t col = c0; col < c1; ++col) {
                double px[3] = {0, 0, 0};
                uint32_t pixel = (uint32_t)((size_t)row * cam.image_w + col);
                for (size_t si = 0; si < spp; ++si) {
                    uint32_t rng = oracle_sample_seed(base_seed, pixel, (uint32_t)si);
                    V3 o, d;
                    primary_ray(&cam, (size_t)row, col, &rng, &o, &d);
                    double c[3];
                    ray_color(&w, &cam, o, d, cam.max_depth, &rng, c, stats ? &mine : NULL, stack);
                    if (samples) {
                        double* q = samples + ((((size_t)row - r0) * W + (col - c0)) * spp + si) * 3;
                        q[0] = c[0]; q[1] = c[1]; q[2] = c[2];
                    }
                    px[0] += c[0]; px[1] += c[1]; px[2] += c[2];
                }
                double inv = 1 / (double)spp; /* pixel_color /= spp: *= (1/spp), rgb.h:76 */
                double* q = rgb + (((size_t)row - r0) * W + (col - c0)) * 3;
                q[0] = px[0] * inv; q[1] = px[1] * inv; q[2] = px[2] * inv;
                mine.samples += spp;
            }
        }
        free(stack);
#pragma omp critical
        {
            total.samples += mine.samples; total.rays += mine.rays; total.nodes_visited += mine.nodes_visited;
            total.sphere_tests += mine.sphere_tests; total.parallelogram_tests += mine.parallelogram_tests;
        }
    }
    if (stats) *stats = total;
    world_free(&w);
    return 0;
}

int oracle_bvh(const crt_material* mats, size_t nm, const crt_object* objs, size_t no,
               uint32_t num_buckets, uint32_t max_prims, crt_bvh_node* nodes, size_t max_nodes,
               size_t* num_nodes, uint32_t* order, size_t max_prims_out, size_t* num_prims) {
    (void)nm;
    World w;
    world_make(mats, objs, no, num_buckets, max_prims, &w);
    *num_nodes = w.nn;
    *num_prims = w.np;
    int rc = 0;
    if (w.nn > max_nodes || w.np > max_prims_out) rc = -2;
    else {
        memcpy(nodes, w.nodes, sizeof(crt_bvh_node) * w.nn);
        memcpy(order, w.order, sizeof(uint32_t) * w.np);
    }
    world_free(&w);
    return rc;
}

int oracle_hits(const crt_material* mats, size_t nm, const crt_object* objs, size_t no,
                const double* rays, size_t n, double t_min, double t_max, crt_hit* out) {
    (void)nm;
    World w;
    world_make(mats, objs, no, 32, 12, &w);
    size_t* stack = (size_t*)malloc(sizeof(size_t) * (w.depth + 2));
    for (size_t i = 0; i < n; ++i) {
        V3 o = ld(rays + 6 * i), d = ld(rays + 6 * i + 3);
        Hit h;
        crt_hit r;
        memset(&r, 0, sizeof r);
        r.prim = -1;
        if (bvh_hit(&w, o, d, t_min, t_max, &h, NULL, stack)) {
            r.t = h.t;
            r.point[0] = h.p.x; r.point[1] = h.p.y; r.point[2] = h.p.z;
            r.normal[0] = h.n.x; r.normal[1] = h.n.y; r.normal[2] = h.n.z;
            r.prim = (int32_t)w.order[h.slot];
            r.front_face = h.front;
            r.material = h.mat;
        }
        out[i] = r;
    }
    free(stack);
    world_free(&w);
    return 0;
}

/* ---- Image::send_as_ppm values (image.h:38-56, rgb.h:10-13, 27-29, 99-115) ------------- */
static volatile double g_gamma = 2; /* runtime exponent: keeps pow(x, 1/gamma) a libm pow call */

static int32_t to_int_x86(double v) { /* static_cast<int> as cvttsd2si */
    if (!(v > -2147483649.0 && v < 2147483648.0)) return INT32_MIN;
    return (int32_t)v;
}

void oracle_ppm_values(const double* rgb, size_t n, int32_t* out) {
    const double gamma = g_gamma, scale = 255 + 0.999999;
    for (size_t i = 0; i < n; ++i) {
        const double r = rgb[3 * i], g = rgb[3 * i + 1], b = rgb[3 * i + 2];
        const double L = 0.2126 * r + 0.7152 * g + 0.0722 * b;
        double c[3] = {r, g, b};
        for (int k = 0; k < 3; ++k) {
            c[k] /= 1 + L;
            out[3 * i + k] = to_int_x86(scale * pow(c[k], 1 / gamma));
        }
    }
}
