/* Plain-C consumer of the C-ABI (include/cfm_*.h): every header compiles as C99 and the library
 * links and answers host-side calls.  Built and run by tests/test_abi.py::test_c_consumer (CPU; no
 * GPU compute).  Prints one line per check; exits non-zero on the first failure. */
#include <stdio.h>
#include <stdlib.h>

#include "cfm_augment.h"
#include "cfm_ctc.h"
#include "cfm_encoder.h"
#include "cfm_joint.h"
#include "cfm_mel.h"
#include "cfm_rnnt_decode.h"
#include "cfm_rnnt_loss.h"
#include "cfm_stream.h"
#include "cfm_train.h"

#define CHECK(cond, msg)                              \
  do {                                                \
    if (!(cond)) {                                    \
      fprintf(stderr, "FAIL: %s\n", msg);             \
      return 1;                                       \
    }                                                 \
    printf("ok: %s\n", msg);                          \
  } while (0)

int main(void) {
  CHECK(cfm_version() == CFM_ABI_VERSION, "cfm_version");
  /* conformer_encoder.py calc_length (subsampling.py:272-282): T = 1000 -> T' = 250, T = 1 -> 1 */
  CHECK(cfm_encoded_length(1000) == 250 && cfm_encoded_length(1) == 1 && cfm_encoded_length(7) == 2,
        "cfm_encoded_length");
  /* invalid arguments come back as status codes with a message, never as a crash */
  CHECK(cfm_spec_mask_rects(NULL, 1, 80, 10, NULL, 1, 0.0f, NULL) == CFM_ERR_INVALID_ARG, "invalid-arg status");
  CHECK(cfm_last_error() != NULL && cfm_last_error()[0] != '\0', "cfm_last_error message");
  cfm_rnnt_decoder* dec = NULL;
  CHECK(cfm_rnnt_decoder_create(0, 640, 1, 0, &dec) == CFM_ERR_INVALID_ARG && dec == NULL, "decoder arg check");
  return 0;
}
