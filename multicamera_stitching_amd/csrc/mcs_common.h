// mcs_common.h -- host-side declarations shared by the plan builder, the runtime binding and the
// C ABI (all compiled with g++; the kernels are a separate gfx950 code object).
#pragma once

#include <stdint.h>

#include "mcs.h"
#include "mcs_kparams.h"

namespace mcs {

int fail(int code, const char *fmt, ...);
const char *last_error();
void clear_error();

void invert3x3_cv(const double *m, double *out);
int build_flat(const mcs_stage_desc *stages, int n_stages, int cam0_w, int cam0_h, int channels,
               int interp, mcs_flat_desc *fd);
void fill_kparams(const mcs_flat_desc &fd, KParams *kp);

}  // namespace mcs
