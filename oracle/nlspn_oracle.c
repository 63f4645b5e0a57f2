/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C CPU restatement of the reference's propagation hot path
 * (XJTUXYC/NLSPN_ECCV20: src/model/nlspnmodel.py:179-381 and the DCNv2 forward
 * it rides on, src/model/deformconv/src/cuda/modulated_deform_im2col_cuda.cuh:24-54,
 * 127-194 + modulated_deform_conv_cuda.cu:19-121).  Only tests/, the smoke() of
 * __graft_entry__.py and bench.py's cpu_baseline leg may load this library, and
 * only as the checker / CPU baseline — never as the thing measured or shipped.
 *
 * Parity pinning (see DESIGN.md "Oracle"): the affinity normalisation, the
 * no-offset branch and the full T-iteration loop are pinned against golden
 * vectors produced by the reference's own Python (tests/golden/gen_golden.py);
 * the DCN (offset) branch has no runnable reference (no CPU DCN in the reference,
 * CUDA extension unbuildable here) and is pinned through the reference's
 * identities: zero offsets == no-offset branch in the interior, integer offsets
 * == shifted reads, zero-offset DCN == conv2d (deformconv/test.py:69-110).
 *
 * Built with -ffp-contract=off so the float path issues the same IEEE operation
 * sequence as written (and as the HIP kernels, which are built the same way).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

enum { ORC_AS = 0, ORC_ASS = 1, ORC_TC = 2, ORC_TGASS = 3 };
#define ORC_PRESERVE 1u
#define ORC_ALWAYS_CLIP 2u

static int orc_threads = 1;

void orc_set_threads(int n) { orc_threads = n < 1 ? 1 : n; }
int orc_get_threads(void) { return orc_threads; }

#define REAL float
#define FN(name) name##_f32
#define TANH tanhf
#define FABS fabsf
#define FLOOR floorf
#include "nlspn_oracle_impl.h"
#undef REAL
#undef FN
#undef TANH
#undef FABS
#undef FLOOR

#define REAL double
#define FN(name) name##_f64
#define TANH tanh
#define FABS fabs
#define FLOOR floor
#include "nlspn_oracle_impl.h"
#undef REAL
#undef FN
#undef TANH
#undef FABS
#undef FLOOR
