// sdf_guard.hpp — exact CSG early-outs for SDF node programs (host side).
#pragma once

#include <stdint.h>

#include <vector>

#include "../../include/rrte_hip.h"

namespace rrte {

// Guard layout inside a decorated program (program-relative indices):
//  * the first node of a guarded right operand B carries i[2] = j + 1, j = the CSG op consuming B;
//  * op node j carries the bound of B in its otherwise unused floats: f[4..6] centre, f[7] radius
//    R, f[8] slope lambda, f[9] the largest |p - centre| the guard may be used at.
// For |p - centre| in [R, f[9]], every value B can return at p is >= lambda * (|p - centre| - R)
// (inflated so that f32 rounding of B's formulas stays inside the margin), so when that lower
// bound alone decides the op (union: bound >= a; smooth union: h(a, bound) == 1; difference:
// -bound <= a; smooth difference: h(-a, bound) == 1) the op's result is exactly its left
// operand and B is not evaluated.  The device takes the early-out only when every active lane
// of the wave may take it (ray_kernels.hpp sdf_guard), so results are bit-identical with guards
// on or off.
constexpr uint32_t kGuardSlot = 2;  // rrte_sdf_node::i[kGuardSlot]

// Rewrites nodes[0..count) in place (count = one program): clears every i[kGuardSlot] and the op
// nodes' guard floats, then adds the guards that pay (min_leaves: 1 = every operand, 2 = operands
// of >= 2 leaves and single leaves of the long formulas, N = operands of >= N leaves).  Returns
// the number of guards added.  Programs the validator accepts only.
uint32_t decorate_sdf_guards(rrte_sdf_node* nodes, uint32_t count, uint32_t min_leaves);

// The scene's node array with every SDF object's program decorated (min_leaves 0: guards off,
// links cleared).  Programs whose node ranges overlap a different program's are left as they are.
std::vector<rrte_sdf_node> decorate_scene_sdf(const rrte_scene_ir* s, uint32_t min_leaves);

}  // namespace rrte
