// The device controller's status word (State::status), shared by the kernels and the host-only
// slot scheduler (slot_sched.h), which includes no HIP header.
#pragma once

#include <stdint.h>

namespace midagma {

enum Status : int32_t {
  ST_RUNNING = 0,
  ST_DONE = 1,          // max_iter reached or checkpoint tolerance met  -> (W, True)
  ST_FAILED = 2,        // left the M-matrix domain at iter 1 or s <= 0.9 -> (W, False)
  ST_LR_UNDERFLOW = 3,  // lr halved below 1e-16                         -> (W, True)
  ST_SINGULAR = 4,      // non-finite inverse                            -> LinAlgError
  ST_NEED_GJ = 5,       // internal: the fast inverse could not run this slot (no usable warm
                        // start, or a log-det is due); the host re-runs it on the GJ path
  ST_HANDOFF_TIMEOUT = 6,  // internal: a bounded in-kernel hand-off wait expired (never expected);
                           // the host resets the hand-off words and raises RuntimeError
};

}  // namespace midagma
