/*
 * opal_hip_bridge.h -- the drop-in boundary on Open MPI's own types: the convertor's
 * fAdvance / fPosition slots served by the MI355X engine (libddt_hip.so).
 *
 * Open MPI has no component framework for datatype engines; the accelerator movers are
 * hard-wired in opal_convertor_prepare_for_{recv,send} (opal_convertor.c:633-635,
 * :677-679) when check_addr reports a device buffer (:593-608).  The reference's own
 * precedent for replacing them after prepare is pack_description_sweep.c:877-965, which
 * overrides convertor->fAdvance.  This bridge does the same: after prepare,
 * opal_hip_bridge_attach() points fAdvance at opal_pack_hip / opal_unpack_hip and
 * fPosition at opal_position_hip.  INTEGRATION.md §1 shows the three-line patch.
 *
 * Built inside an Open MPI tree, the real opal headers define the types; here
 * opal_layout.h restates their LP64 layout with compile-time offset checks.
 */
#ifndef OPAL_HIP_BRIDGE_H
#define OPAL_HIP_BRIDGE_H

#ifndef OPAL_CONVERTOR_H_HAS_BEEN_INCLUDED
#include "opal_layout.h"
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* convertor_advance_fct_t (opal_convertor.h:102-103); replaces opal_pack_accelerator_simple
 * (opal_datatype_pack_accelerator.c:161-295, prototype opal_datatype_prototypes.h:44-45).
 * Packs from conv->bConverted into iov[0..*out_size); rewrites iov_len, *out_size and
 * *max_data; advances bConverted; returns 1 and sets CONVERTOR_COMPLETED at the end of the
 * message, 0 when more remains, < 0 on error.  Never splits a predefined element of the
 * description (_pack_accelerator.c:52-58).  With CONVERTOR_ACCELERATOR_ASYNC the kernels are
 * queued on conv->stream and the call returns without synchronising. */
int32_t opal_pack_hip(opal_convertor_t *conv, struct iovec *iov, uint32_t *out_size, size_t *max_data);
/* replaces opal_unpack_accelerator_simple (opal_datatype_unpack_accelerator.c:210-368);
 * accepts any byte window, mid-element splits included (:344-352). */
int32_t opal_unpack_hip(opal_convertor_t *conv, struct iovec *iov, uint32_t *out_size, size_t *max_data);
/* convertor_position_fct_t (opal_convertor.h:104), called by opal_convertor_set_position
 * (:357-394) for a position inside the stream; replaces opal_convertor_position_generic
 * (opal_convertor.c:445-471).  A send convertor lands on the predefined-element boundary of
 * use_desc at or below *position and returns it there (:465-469); a receive convertor takes
 * the byte.  The engine resumes from the byte position alone, so this records it
 * (bConverted) and clears the descriptor stack. */
int32_t opal_position_hip(opal_convertor_t *conv, size_t *position);

/* Post-prepare hook: for a homogeneous accelerator convertor (CONVERTOR_ACCELERATOR set by
 * check_addr) import conv->use_desc once per datatype and install the three functions above.
 * Returns OPAL_SUCCESS, or OPAL_ERR_NOT_SUPPORTED leaving the convertor untouched (host buffer,
 * heterogeneous), or < 0 when the description cannot be imported. */
int opal_hip_bridge_attach(opal_convertor_t *conv);

/* Commit hook: call at the end of opal_datatype_commit (opal_datatype_optimize.c:1739-1782, after
 * the fake END_LOOP is set) so a large description -- at least OPAL_HIP_BRIDGE_COMMIT_IMPORT_MIN
 * opt_desc entries -- is imported (and a large index list gets its device tables) inside
 * MPI_Type_commit, where Open MPI pays its own optimizer pass, instead of at the first prepare of
 * a message; smaller descriptions import at first use in microseconds.  The convertor's use_desc
 * of a homogeneous convertor is &dt->opt_desc (OPAL_CONVERTOR_PREPARE, opal_convertor.c:533), so
 * attach then finds the entry.  Returns OPAL_SUCCESS or the import's error (the datatype stays
 * usable: attach retries). */
#define OPAL_HIP_BRIDGE_COMMIT_IMPORT_MIN 65536
int opal_hip_bridge_datatype_commit(const opal_datatype_t *dt);

/* Drop the cached import of `dt`; call from opal_datatype_destruct (opal_datatype_create.c:61-91)
 * so a datatype freed and reallocated at the same address is never served a stale plan. */
void opal_hip_bridge_datatype_destruct(const opal_datatype_t *dt);
/* Drop every cached import (opal_datatype_finalize). */
void opal_hip_bridge_finalize(void);
/* Counters for tests: out[0] = cached types, out[1] = imports so far, out[2] = cache hits,
 * out[3] = stale entries replaced (fingerprint mismatch at the same address). */
void opal_hip_bridge_stats(size_t *out4);
/* Layout self-description of the compiled bridge, for the harness that builds opal-shaped
 * objects: out[0..7] = sizeof(opal_datatype_t), offsetof(opal_datatype_t, opt_desc),
 * sizeof(opal_convertor_t), offsetof(opal_convertor_t, bConverted), offsetof(.., flags),
 * offsetof(.., fPosition), offsetof(.., stream), sizeof(dt_elem_desc_t). */
void opal_hip_bridge_layout(size_t *out8);

#ifdef __cplusplus
}
#endif
#endif /* OPAL_HIP_BRIDGE_H */
