// sdf_guard.hip — host analysis of SDF node programs: a conservative bound per CSG subtree and
// the guards that let a wave skip the right operand of a union / difference exactly
// (sdf_guard.hpp).  The bounds follow the build-defined leaf formulas of ray_kernels.hpp
// sdf_leaf; each case states why value(p) >= lambda * (|q| - R) for |q| >= R,
// q = p - centre.
#include "sdf_guard.hpp"

#include <algorithm>
#include <cmath>
#include <vector>

namespace rrte {
namespace {

struct Bound {
    bool ok = false;
    double c[3] = {0, 0, 0};
    double R = 0, lam = 1;
};

struct Sub {
    uint32_t start;   // first node of the subtree
    uint32_t leaves;  // leaves in it
    bool clean;       // no deformer / POP_POINT inside (every leaf sees the point of `start`)
    Bound b;
};

bool fin(double v) { return std::isfinite(v); }

Bound leaf_bound(const rrte_sdf_node& n) {
    Bound b;
    const float* f = n.f;
    for (int k = 0; k < 7; ++k)
        if (!fin(f[k])) return b;
    b.c[0] = f[0], b.c[1] = f[1], b.c[2] = f[2];
    auto nonneg = [&](std::initializer_list<int> ks) {
        for (int k : ks)
            if (!(f[k] >= 0.0f)) return false;
        return true;
    };
    switch (n.op) {
    case RRTE_SDF_SPHERE:  // |q| - r
        if (!nonneg({3})) return b;
        b.R = f[3];
        break;
    case RRTE_SDF_BOX:  // exact box distance >= |q| - half diagonal
        if (!nonneg({4, 5, 6})) return b;
        b.R = 0.5 * std::sqrt((double)f[4] * f[4] + (double)f[5] * f[5] + (double)f[6] * f[6]);
        break;
    case RRTE_SDF_CYLINDER:  // exact capped cylinder
    case RRTE_SDF_CONE:      // exact capped cone: profile points lie within hypot(r, h/2) of the centre
        if (!nonneg({3, 4})) return b;
        b.R = std::hypot((double)f[3], 0.5 * f[4]);
        break;
    case RRTE_SDF_PRISM: {
        // max(|qz| - d/2, max(0.866|qx| + 0.5qy, -qy) - sy/4) >= max_i(n_i.q) - max(d/2, sy/4); the
        // unit normals (0,0,+-1), (+-0.866,0.5,0), (0,-1,0) give max_i(n_i.u) >= 1/sqrt(5) for every
        // unit u (worst case |u_xy| = 2/sqrt(5): 0.5|u_xy| = |u_z|), so value >= lam(|q| - o/lam).
        if (!nonneg({5, 6})) return b;
        b.lam = 0.44;
        b.R = std::max(0.5 * f[6], 0.25 * f[5]) / b.lam;
        break;
    }
    case RRTE_SDF_TORUS:  // |(|q.xz| - R, q.y)| - r >= |q| - R - r (triangle inequality)
    case RRTE_SDF_RING:   // the same in XY
        if (!nonneg({3, 4})) return b;
        b.R = (double)f[3] + f[4];
        break;
    case RRTE_SDF_TUBE: {
        // exact 2-D box distance in (radius, y) about (mid, 0): >= |(rad - mid, y)| - |(half, h/2)|
        // >= |q| - mid - |(half, h/2)|
        if (!nonneg({3, 4, 5}) || !(f[3] >= f[4])) return b;
        const double mid = 0.5 * ((double)f[3] + f[4]), half = 0.5 * ((double)f[3] - f[4]);
        b.R = mid + std::hypot(half, 0.5 * f[5]);
        break;
    }
    case RRTE_SDF_CAPSULE:  // exact: segment of half-length h/2, radius r
        if (!nonneg({3, 4})) return b;
        b.R = (double)f[3] + 0.5 * f[4];
        break;
    case RRTE_SDF_ELLIPSOID: {
        // k0 = |q/r| >= |q|/rmax >= 1 outside the rmax ball, k1 = |q/r^2| <= |q|/rmin^2, and k0(k0-1)
        // grows for k0 >= 1/2: k0(k0-1)/k1 >= (rmin/rmax)^2 (|q| - rmax)
        if (!(f[4] > 0.0f && f[5] > 0.0f && f[6] > 0.0f)) return b;
        const double rmin = std::min({(double)f[4], (double)f[5], (double)f[6]});
        const double rmax = std::max({(double)f[4], (double)f[5], (double)f[6]});
        b.lam = (rmin / rmax) * (rmin / rmax);
        b.R = rmax;
        break;
    }
    default:
        return b;
    }
    b.ok = fin(b.R) && b.lam > 0.0;
    return b;
}

// Smallest sphere around two spheres (slope = the smaller one: lam_i (|p-c_i| - R_i) >= lam (|p-c| - R)
// once p is outside the merged sphere).
Bound merge(const Bound& x, const Bound& y) {
    Bound m;
    if (!x.ok || !y.ok) return m;
    m.ok = true;
    m.lam = std::min(x.lam, y.lam);
    const double d = std::sqrt((x.c[0] - y.c[0]) * (x.c[0] - y.c[0]) + (x.c[1] - y.c[1]) * (x.c[1] - y.c[1]) +
                               (x.c[2] - y.c[2]) * (x.c[2] - y.c[2]));
    if (d + y.R <= x.R) {
        std::copy(x.c, x.c + 3, m.c);
        m.R = x.R;
    } else if (d + x.R <= y.R) {
        std::copy(y.c, y.c + 3, m.c);
        m.R = y.R;
    } else {
        m.R = 0.5 * (d + x.R + y.R);
        const double t = d > 0 ? (m.R - x.R) / d : 0.0;
        for (int k = 0; k < 3; ++k) m.c[k] = x.c[k] + (y.c[k] - x.c[k]) * t;
        m.R *= 1.0 + 1e-12;
    }
    return m;
}

// Leaf cost class: single leaves are worth a guard only when their formula is long.
bool costly_leaf(uint32_t op) {
    return op == RRTE_SDF_CONE || op == RRTE_SDF_ELLIPSOID || op == RRTE_SDF_TUBE || op == RRTE_SDF_TORUS ||
           op == RRTE_SDF_RING || op == RRTE_SDF_CYLINDER;
}

}  // namespace

uint32_t decorate_sdf_guards(rrte_sdf_node* nodes, uint32_t count, uint32_t min_leaves) {
    for (uint32_t i = 0; i < count; ++i) {
        nodes[i].i[kGuardSlot] = 0u;
        if (nodes[i].op >= RRTE_SDF_UNION && nodes[i].op <= RRTE_SDF_SMOOTH_INTERSECTION)
            for (int k = 4; k < 10; ++k) nodes[i].f[k] = 0.0f;
    }
    std::vector<Sub> st;
    std::vector<uint32_t> deform_at;  // node index of each open deformer
    uint32_t added = 0;
    for (uint32_t j = 0; j < count; ++j) {
        const rrte_sdf_node& n = nodes[j];
        const uint32_t op = n.op;
        if (op >= RRTE_SDF_SPHERE && op <= RRTE_SDF_ELLIPSOID) {
            st.push_back(Sub{j, 1u, true, leaf_bound(n)});
        } else if (op >= RRTE_SDF_UNION && op <= RRTE_SDF_SMOOTH_INTERSECTION) {
            if (st.size() < 2) return added;  // not a validated program
            const Sub B = st.back();
            st.pop_back();
            const Sub A = st.back();
            st.pop_back();
            const double k = n.f[0];
            const bool smooth = op >= RRTE_SDF_SMOOTH_UNION;
            const bool k_ok = !smooth || (fin(k) && k > 0.0);
            Sub r{A.start, A.leaves + B.leaves, A.clean && B.clean, Bound{}};
            if (k_ok && r.clean) {
                switch (op) {
                case RRTE_SDF_UNION:
                    r.b = merge(A.b, B.b);
                    break;
                case RRTE_SDF_SMOOTH_UNION:  // smin >= min - k/4
                    r.b = merge(A.b, B.b);
                    if (r.b.ok) r.b.R += k / (4.0 * r.b.lam);
                    break;
                case RRTE_SDF_DIFFERENCE:
                case RRTE_SDF_SMOOTH_DIFFERENCE:  // max(a, -b) >= a;  -smin(-a, b) >= max(a, -b)
                    r.b = A.b;
                    break;
                default:  // intersections: >= max(a, b)
                    r.b = (A.b.ok && (!B.b.ok || A.b.R / A.b.lam <= B.b.R / B.b.lam)) ? A.b : B.b;
                    break;
                }
            }
            // guard B: unions and differences whose left operand alone can decide the result
            const bool guardable_op = op == RRTE_SDF_UNION || op == RRTE_SDF_SMOOTH_UNION ||
                                      op == RRTE_SDF_DIFFERENCE || op == RRTE_SDF_SMOOTH_DIFFERENCE;
            const bool worth = B.leaves >= min_leaves ||
                               (min_leaves == 2u && B.leaves == 1u && costly_leaf(nodes[B.start].op));
            bool clean = B.clean;
            for (uint32_t x = B.start; x < j && clean; ++x) clean = nodes[x].op < RRTE_SDF_BEND;
            if (guardable_op && k_ok && clean && B.b.ok && worth) {
                const double cn = std::sqrt(B.b.c[0] * B.b.c[0] + B.b.c[1] * B.b.c[1] + B.b.c[2] * B.b.c[2]);
                // margin: the f32 formulas of B and the guard's own distance are within ~1e-5 of
                // exact for points inside the usable range; the margin is 1e-3 + 1e-4 (R + |c|).
                const double R = B.b.R + 1e-3 + 1e-4 * (B.b.R + cn);
                const double lam = B.b.lam * (1.0 - 1e-4);
                const double smax = 16.0 * (B.b.R + 1.0);
                if (fin(R) && R < 1e6 && cn < 1e6) {
                    rrte_sdf_node& g = nodes[j];
                    g.f[4] = (float)B.b.c[0];
                    g.f[5] = (float)B.b.c[1];
                    g.f[6] = (float)B.b.c[2];
                    // round the radius up and the slope down so the f32 copies stay conservative
                    g.f[7] = std::nextafter((float)R, INFINITY);
                    g.f[8] = std::nextafter((float)lam, 0.0f);
                    g.f[9] = (float)smax;
                    nodes[B.start].i[kGuardSlot] = j + 1u;
                    ++added;
                }
            }
            st.push_back(r);
        } else if (op >= RRTE_SDF_BEND && op <= RRTE_SDF_WAVE) {
            deform_at.push_back(j);
        } else if (op == RRTE_SDF_POP_POINT) {
            if (deform_at.empty()) return added;
            const uint32_t d = deform_at.back();
            deform_at.pop_back();
            // values pushed since the deformer were evaluated at the deformed point: their bounds
            // do not hold in the outer point space, and their ranges begin at the deformer
            bool first = true;
            for (Sub& s : st)
                if (s.start > d) {
                    s.clean = false;
                    s.b.ok = false;
                    if (first) s.start = d;
                    first = false;
                }
        }
    }
    return added;
}

}  // namespace rrte

namespace rrte {

std::vector<rrte_sdf_node> decorate_scene_sdf(const rrte_scene_ir* s, uint32_t min_leaves) {
    std::vector<rrte_sdf_node> out(s->sdf_nodes, s->sdf_nodes + s->num_sdf_nodes);
    for (rrte_sdf_node& n : out) n.i[kGuardSlot] = 0u;  // the caller's i[2] carries no meaning
    // distinct program ranges; two different ranges that overlap would read each other's
    // (program-relative) links, so such programs stay undecorated
    std::vector<std::pair<uint32_t, uint32_t>> ranges;
    for (uint32_t i = 0; i < s->num_prims; ++i) {
        const rrte_prim& pr = s->prims[i];
        if (pr.kind != RRTE_PRIM_SDF || pr.sdf_count == 0) continue;
        if ((uint64_t)pr.sdf_first + pr.sdf_count > s->num_sdf_nodes) continue;
        const std::pair<uint32_t, uint32_t> r{pr.sdf_first, pr.sdf_count};
        if (std::find(ranges.begin(), ranges.end(), r) == ranges.end()) ranges.push_back(r);
    }
    for (size_t a = 0; a < ranges.size(); ++a) {
        const uint32_t f0 = ranges[a].first, e0 = f0 + ranges[a].second;
        bool overlap = false;
        for (size_t b = 0; b < ranges.size() && !overlap; ++b) {
            if (a == b) continue;
            const uint32_t f1 = ranges[b].first, e1 = f1 + ranges[b].second;
            overlap = f0 < e1 && f1 < e0;
        }
        if (overlap || !min_leaves) continue;
        decorate_sdf_guards(out.data() + f0, ranges[a].second, min_leaves);
    }
    return out;
}

}  // namespace rrte
