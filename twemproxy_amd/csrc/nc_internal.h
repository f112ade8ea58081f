/* Internal declarations shared between the C host layer and the HIP launch layer. */
#ifndef NC_INTERNAL_H
#define NC_INTERNAL_H

#include "nc_gpuhash.h"
#include "nc_gpuhash_synth.h"
#include "nc_synth_core.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Validate a spec and resolve it into a plan; NC_ERROR (errno EINVAL) on a bad spec. */
__attribute__((visibility("hidden")))
rstatus_t nc_synth_make_plan(const struct nc_synth_spec *spec, struct nc_synth_plan *plan);

#ifdef __cplusplus
}
#endif

#endif
