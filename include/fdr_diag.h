/*
 * fdr_diag.h -- diagnostics of libfdr.so, OUTSIDE the drop-in boundary (include/fdr.h).
 *
 * Measurement and A/B facilities the benchmark and the tools/ scripts use; nothing a caller of the reference's
 * interfaces needs, and no result of the compute calls depends on them except where stated (the replay switch
 * selects between two bit-identical forms).  Same conventions as fdr.h: int error codes, host-side state only.
 */
#ifndef FDR_DIAG_H_
#define FDR_DIAG_H_

#include "fdr.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Opt-in phase timing of fdr_impala_rollout (per context; the fdr_impala_* forms act on the default context; not
 * thread-safe): when enabled, HIP events are recorded between the step-loop launches; fdr_ctx_impala_profile_read
 * waits for the last profiled rollout and returns HOST ms[3] = summed conv-stack / core (fc+LSTM+head) /
 * entropy-replay kernel time.  Used by bench.py for the live roofline figure. */
int fdr_ctx_impala_profile(fdr_ctx* ctx, int32_t enable);
int fdr_ctx_impala_profile_read(fdr_ctx* ctx, double* ms);
int fdr_impala_profile(int32_t enable);
int fdr_impala_profile_read(double* ms);

/* Phase clocks: subsequent fdr_impala_rollout launches write s_memtime clocks of conv workgroup 0 at its phase
 * boundaries into the DEVICE buffer buf (u64[128]: stage / block / entry-band boundaries at 0..63, diagnostics
 * builds also 64..127; overwritten each step); NULL = off.  tools/impala_phases_h2.py. */
int fdr_ctx_impala_debug_clock(fdr_ctx* ctx, uint64_t* buf);
int fdr_impala_debug_clock(uint64_t* buf);

/* Entropy replay of fdr_impala_rollout (default on): 1 = the x W_ih^T half of the replayed LSTM gates is one MFMA
 * GEMM per lane (pair) over 64-step chunks; 0 = every replay step streams [W_ih | W_hh] (the step kernel's form).
 * Both give bit-identical gates (tests/test_gpu_impala.py). */
int fdr_ctx_set_replay_gemm(fdr_ctx* ctx, int32_t on);
int fdr_impala_set_replay_gemm(int32_t on);

#ifdef __cplusplus
}
#endif
#endif /* FDR_DIAG_H_ */
