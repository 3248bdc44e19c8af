/*
 * cfm_augment.h — C-ABI of the on-device spectrogram augmentation (libcfm.so), SURVEY §8 row f4:
 * the training-time step between the mel front end and the encoder.
 *
 * Replaces the per-utterance host loops and slice assignments of
 *   SpecAugment.forward()   (spectr_augment.py:80-105: freq / time masks, in place)
 *   SpecCutout.forward()    (spectr_augment.py:138-152: rectangles, in place)
 *   SpecShot.forward()      (spectr_augment.py:177-184: keep where 1 - U(0,1) > mask_ratio)
 * as driven by SpectrogramAugmentation.forward() (audio_preprocessing.py:511-521).
 *
 * Mask geometry is drawn on the host with the reference's own random.Random call sequence (so a
 * seeded rng reproduces the reference's masks exactly) and handed over as one table of rectangles;
 * a single launch then writes every rectangle of every utterance.  SpecShot draws its per-element
 * uniforms on the device from a counter-based hash of (seed, element index); the reference draws
 * them from torch's CPU generator, so SpecShot matches it in distribution, not bit for bit.
 *
 * Conventions as in cfm_encoder.h: device pointers, fp32, status codes + cfm_last_error(),
 * stream-ordered (void* = hipStream_t), no host synchronisation, nothing allocated.
 */
#ifndef CFM_AUGMENT_H_
#define CFM_AUGMENT_H_

#include <stddef.h>
#include <stdint.h>

#include "cfm_encoder.h"

#ifdef __cplusplus
extern "C" {
#endif

/* spec (B, F, T) fp32, in place.  rects (B, n, 4) int32 on the device: [f0, f1, t0, t1) per
 * rectangle, Python-slice semantics (bounds clamped to [0, F] x [0, T]; empty rectangles are
 * no-ops).  spec[b, f0:f1, t0:t1] = value for every rectangle of utterance b. */
cfm_status cfm_spec_mask_rects(float* spec, int B, int F, int T, const int32_t* rects, int n, float value,
                               void* stream);

/* out = in * (1 - u > mask_ratio), u = hash-uniform in [0, 1) of (seed, b*F*T + f*T + t), for the
 * n = B*F*T elements; out may alias in. */
cfm_status cfm_spec_shot(const float* in, float* out, int64_t n, float mask_ratio, uint64_t seed, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CFM_AUGMENT_H_ */
