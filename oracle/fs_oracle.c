/* oracle/fs_oracle.c -- test infrastructure, never the product path.
 *
 * CPU restatement of the score the full-sort kernels rank by (reference
 * src/common/trainer.py:509-528 via src/models/*.py full_sort_predict: the user rows
 * times the item rows, masked train items set to -1e10, topk): the exact f32 score of
 * the rsx kernels is an fmaf chain over d in order (csrc/fullsort.hip exact_dot,
 * score_dense), restated here with C's fmaf so the tests can anchor the screened
 * kernel's top-k on the CPU rather than on another kernel of the same library.
 * Built by __graft_entry__.build() / rsx.build into oracle/_build/libfsoracle.so.
 */
#include <math.h>
#include <stdint.h>

/* out[b * ni + i] = fmaf chain over c of U[users[b]][c] * I[i][c] (c = 0 .. d-1) */
void rsx_oracle_fmaf_scores(const float* U, const int64_t* users, int64_t nb, const float* I, int64_t ni, int32_t d,
                            float* out) {
#pragma omp parallel for schedule(dynamic, 4)
    for (int64_t b = 0; b < nb; ++b) {
        const float* u = U + users[b] * (int64_t)d;
        float* o = out + b * ni;
        for (int64_t i = 0; i < ni; ++i) {
            const float* v = I + i * (int64_t)d;
            float acc = 0.f;
            for (int32_t c = 0; c < d; ++c) acc = fmaf(u[c], v[c], acc);
            o[i] = acc;
        }
    }
}
