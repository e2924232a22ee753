/*
 * catseg_hip_tuning.h — diagnostics / A-B entry of libcatseg_hip.so.  NOT part of the product
 * C ABI (include/catseg_hip.h): a reference-side caller never needs it.  Every kernel family
 * picks its tiling / variant automatically; these knobs force an alternative for same-process
 * A/B timing (tools/) and for the tests that prove every alternative computes the same bits.
 * Knobs are process-wide and read at launch time (so at hipGraph capture).
 */
#ifndef CATSEG_HIP_TUNING_H
#define CATSEG_HIP_TUNING_H
#ifdef __cplusplus
extern "C" {
#endif
/* Set knob `name` to `value`; returns 0, or -1 for an unknown name.  Known names:
 * catseg_tuning_list(). */
int catseg_tuning_set(const char* name, int value);
/* Current value of knob `name` into *value; 0, or -1 for an unknown name. */
int catseg_tuning_get(const char* name, int* value);
/* Comma-separated names of every registered knob (static storage). */
const char* catseg_tuning_list(void);
#ifdef __cplusplus
}
#endif
#endif /* CATSEG_HIP_TUNING_H */
