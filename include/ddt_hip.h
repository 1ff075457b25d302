/*
 * ddt_hip.h -- C ABI of libddt_hip.so, an MI355X-native MPI derived-datatype
 * pack/unpack engine that sits behind Open MPI's datatype/convertor API.
 *
 * Every entry point uses plain pointers and sizes.  Each one names the Open MPI
 * interface it replaces (paths relative to the Open MPI source tree).  The
 * convertor functions keep the reference's argument meaning and return codes:
 * pack/unpack return 1 when the whole message has been converted, 0 when more
 * fragments remain, and a negative code on error (opal_convertor.h:179-196).
 *
 * Buffers: the user buffer handed to prepare_for_send/recv must be device
 * memory (hipMalloc / hipMallocManaged) -- this is the accelerator slot of the
 * convertor, selected by opal_convertor_prepare_for_{send,recv} when
 * check_addr reports a device pointer (opal_convertor.c:593-608).  The packed
 * iovec buffers may be device or host memory: pinned host iovecs are read or
 * written by the kernel itself over PCIe, pageable ones are staged through HBM
 * slots with hipMemcpyAsync on a copy stream.
 */
#ifndef DDT_HIP_H
#define DDT_HIP_H

#include <stddef.h>
#include <stdint.h>
#include <sys/uio.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- return codes (mirror OPAL_SUCCESS / OPAL_ERR_* sign convention) ---- */
#define DDT_SUCCESS 0
#define DDT_ERROR (-1)
#define DDT_ERR_OUT_OF_RESOURCE (-2)
#define DDT_ERR_BAD_PARAM (-5)
#define DDT_ERR_NOT_COMMITTED (-6)
#define DDT_ERR_NOT_DEVICE (-7)     /* user buffer is not device memory */
#define DDT_ERR_HIP (-8)            /* a HIP runtime call failed */
#define DDT_ERR_TRUNCATE (-9)       /* MPI_ERR_TRUNCATE analogue for ddt_pack/ddt_unpack */
#define DDT_ERR_NOT_SUPPORTED (-10)
#define DDT_ERR_VALUE_OUT_OF_BOUNDS (-11) /* MPI_Get_elements: the bytes end inside an element */

/* ---- predefined type ids: identical to OPAL_DATATYPE_* (opal_datatype_internal.h:71-99) ---- */
#define DDT_INT1 4
#define DDT_INT2 5
#define DDT_INT4 6
#define DDT_INT8 7
#define DDT_INT16 8
#define DDT_UINT1 9
#define DDT_UINT2 10
#define DDT_UINT4 11
#define DDT_UINT8 12
#define DDT_UINT16 13
#define DDT_FLOAT2 14
#define DDT_FLOAT4 15
#define DDT_FLOAT8 16
#define DDT_FLOAT12 17
#define DDT_FLOAT16 18
#define DDT_SHORT_FLOAT_COMPLEX 19
#define DDT_FLOAT_COMPLEX 20
#define DDT_DOUBLE_COMPLEX 21
#define DDT_LONG_DOUBLE_COMPLEX 22
#define DDT_BOOL 23
#define DDT_WCHAR 24
#define DDT_LONG 25
#define DDT_UNSIGNED_LONG 26
#define DDT_FLOAT128_COMPLEX 27

/* ---- datatype flags (values of OPAL_DATATYPE_FLAG_*, opal_datatype.h:80-105) ---- */
#define DDT_FLAG_PREDEFINED 0x0002u
#define DDT_FLAG_COMMITTED 0x0004u
#define DDT_FLAG_OVERLAP 0x0008u
#define DDT_FLAG_CONTIGUOUS 0x0010u
#define DDT_FLAG_NO_GAPS 0x0020u
#define DDT_FLAG_USER_LB 0x0040u
#define DDT_FLAG_USER_UB 0x0080u
#define DDT_FLAG_DATA 0x0100u

#define DDT_ORDER_C 0
#define DDT_ORDER_FORTRAN 1
/* MPI_DISTRIBUTE_* (mpi.h.in:595-598) */
#define DDT_DISTRIBUTE_BLOCK 0
#define DDT_DISTRIBUTE_CYCLIC 1
#define DDT_DISTRIBUTE_NONE 2
#define DDT_DISTRIBUTE_DFLT_DARG (-1)

typedef struct ddt_datatype ddt_datatype_t;
typedef struct ddt_convertor ddt_convertor_t;

/* ================= datatype construction (ompi/datatype/ompi_datatype.h:217-284) ================= */

/* Predefined type handle (opal_datatype_basicDatatypes[id], opal_datatype.h:216-248). Never freed.
 * ids 4..27 are the basic types; 2 / 3 are the MPI_LB / MPI_UB bound markers (size 0; a constructor
 * that adds one only moves the lower / upper bound to its displacement, opal_datatype_add.c:158-186). */
const ddt_datatype_t *ddt_predefined(int id);

/* ompi_datatype_create_contiguous (ompi_datatype_create_contiguous.c:31-44) */
int ddt_type_create_contiguous(size_t count, const ddt_datatype_t *oldtype, ddt_datatype_t **newtype);
/* ompi_datatype_create_vector / _hvector (ompi_datatype_create_vector.c:32-88); hvector stride in bytes */
int ddt_type_create_vector(size_t count, size_t blocklen, ptrdiff_t stride,
                           const ddt_datatype_t *oldtype, ddt_datatype_t **newtype);
int ddt_type_create_hvector(size_t count, size_t blocklen, ptrdiff_t stride_bytes,
                            const ddt_datatype_t *oldtype, ddt_datatype_t **newtype);
/* ompi_datatype_create_indexed / _hindexed (ompi_datatype_create_indexed.c:35-114) */
int ddt_type_create_indexed(size_t count, const size_t *blocklens, const ptrdiff_t *disps,
                            const ddt_datatype_t *oldtype, ddt_datatype_t **newtype);
int ddt_type_create_hindexed(size_t count, const size_t *blocklens, const ptrdiff_t *disps_bytes,
                             const ddt_datatype_t *oldtype, ddt_datatype_t **newtype);
/* ompi_datatype_create_indexed_block / _hindexed_block (ompi_datatype_create_indexed.c:117-183) */
int ddt_type_create_indexed_block(size_t count, size_t blocklen, const ptrdiff_t *disps,
                                  const ddt_datatype_t *oldtype, ddt_datatype_t **newtype);
int ddt_type_create_hindexed_block(size_t count, size_t blocklen, const ptrdiff_t *disps_bytes,
                                   const ddt_datatype_t *oldtype, ddt_datatype_t **newtype);
/* ompi_datatype_create_struct (ompi_datatype_create_struct.c:32-98); disps in bytes */
int ddt_type_create_struct(size_t count, const size_t *blocklens, const ptrdiff_t *disps,
                           const ddt_datatype_t *const *types, ddt_datatype_t **newtype);
/* ompi_datatype_create_subarray (ompi_datatype_create_subarray.c:32-112) */
int ddt_type_create_subarray(int ndims, const size_t *sizes, const size_t *subsizes,
                             const size_t *starts, int order, const ddt_datatype_t *oldtype,
                             ddt_datatype_t **newtype);
/* ompi_datatype_create_darray (ompi_datatype_create_darray.c:187-312): the block / cyclic /
 * none distribution of a `ndims`-dimensional global array over a process grid, for `rank`
 * of `size`; gsizes are counts (big-count form). */
int ddt_type_create_darray(int size, int rank, int ndims, const size_t *gsizes, const int *distribs,
                           const int *dargs, const int *psizes, int order,
                           const ddt_datatype_t *oldtype, ddt_datatype_t **newtype);
/* ompi_datatype_create_resized (ompi_datatype.h:270-284) */
int ddt_type_create_resized(const ddt_datatype_t *oldtype, ptrdiff_t lb, ptrdiff_t extent,
                            ddt_datatype_t **newtype);
/* ompi_datatype_duplicate (ompi_datatype_create.c:115-145) */
int ddt_type_dup(const ddt_datatype_t *oldtype, ddt_datatype_t **newtype);
/* opal_datatype_commit (opal_datatype_optimize.c:1739-1782): freezes the type map, derives
 * the reference's opt_desc from it (ddt_type_to_opal_opt_desc) and builds the device plan
 * lazily on first use. */
int ddt_type_commit(ddt_datatype_t *type);
/* The device state a committed type's first move would build: for a large index list of small
 * blocks (>= 1 Mi, the address-ordered engine) its lists and address-ordered tables, on the
 * library-private stream of the current device, which the type's plan is then bound to.
 * ddt_type_commit calls it for such types and the opal bridge at import, so the cost lands where
 * Open MPI pays its own (opal_datatype_commit), not in the first pack of a message.  A no-op for
 * other types and without a device. */
int ddt_type_prepare_device(ddt_datatype_t *type);
/* ompi_datatype_destroy / OBJ_RELEASE; predefined handles are ignored.  Never waits: the type's
 * device memory goes back to the engine's pool behind events recorded on every stream its work
 * was queued on, so those streams must still exist (HIP cannot tell a destroyed stream handle,
 * using one is undefined); work enqueued inside a stream capture keeps its memory for the graph. */
int ddt_type_destroy(ddt_datatype_t **type);

/* ---- queries (opal_datatype.h:290-330) ---- */
int ddt_type_size(const ddt_datatype_t *type, size_t *size);
int ddt_type_get_extent(const ddt_datatype_t *type, ptrdiff_t *lb, ptrdiff_t *extent);
int ddt_type_get_true_extent(const ddt_datatype_t *type, ptrdiff_t *true_lb, ptrdiff_t *true_extent);
uint32_t ddt_type_flags(const ddt_datatype_t *type);
/* out[0..7] = size, lb, ub, true_lb, true_ub, align, flags, nbElems */
int ddt_type_info(const ddt_datatype_t *type, int64_t *out8);
/* Committed metadata of opal_datatype_t (opal_datatype.h:172-212): out[0] = stack_depth (the
 * deeper LOOP nesting of desc and opt_desc, opal_datatype_optimize.c:222-261, :1777), out[1] =
 * bdt_used (predefined ids present, opal_datatype_add.c:163,175,306), out[2] = the optimizer's
 * flags (OPAL_DATATYPE_OPTIMIZED_RESTRICTED), out[3] = 1 once committed.  What
 * opt_desc_equiv.c:223-276 reads to recompute a corpus type's traits. */
int ddt_type_commit_info(const ddt_datatype_t *type, int64_t *out4);
/* MPI_Pack / MPI_Unpack count consolidation: ompi_datatype_consolidate_create
 * (ompi/datatype/ompi_datatype_create_contiguous.c:119-180).  For count >= the threshold (MCA
 * ompi_datatype_consolidate_threshold, default 250; ddt_tune("consolidate")) and a type with gaps,
 * *out = contiguous(count, old) whose opt_desc is ONE loop of count over old's opt_desc,
 * re-optimized on that loop only (opal_datatype_optimize_from_contiguous,
 * opal_datatype_optimize.c:1480-1573) -- committed, owned by the caller; *out = NULL where the
 * reference keeps (count, old).  Same packed bytes; its element boundaries (send positions, pack
 * fragments) are the consolidated description's, as in MPI_Pack. */
int ddt_type_consolidate(const ddt_datatype_t *old, size_t count, ddt_datatype_t **out);

/* Import a committed Open MPI description: `desc` is the opal_datatype_t::opt_desc
 * (or ::desc) array of `used` dt_elem_desc_t entries, 32 bytes each, layout of
 * opal_datatype_internal.h:119-160.  Bounds are copied from the opal_datatype_t.
 * This is the bridge a convertor plug-in uses to hand its type map to the engine. */
int ddt_type_from_opal_desc(const void *desc, size_t used, size_t size, ptrdiff_t lb, ptrdiff_t ub,
                            ptrdiff_t true_lb, ptrdiff_t true_ub, ddt_datatype_t **newtype);

/* The inverse, for tests and tools: the uncommitted type map of `type` as the
 * opal_datatype_t::desc opal_datatype_add would have built (opal_datatype_add.c:307-431:
 * DATA entries, LOOP/END_LOOP pairs as CREATE_LOOP_START/END write them,
 * opal_datatype_internal.h:171-189), without the END_LOOP sentinel.  Returns the entry count,
 * or minus the count needed when `cap` entries do not fit. */
int64_t ddt_type_to_opal_desc(const ddt_datatype_t *type, void *out, size_t cap);

/* opal_datatype_t::opt_desc of `type` as opal_datatype_commit derives it from that desc
 * (opal_datatype_optimize.c:1739-1782, restated in ddt_optimize.cpp: mixed-type regions re-typed
 * to UINT8/4/2/1 carriers, :581-630), without the sentinel; *flags (optional) gets
 * OPAL_DATATYPE_OPTIMIZED_RESTRICTED (0x10000) when a region was re-typed.  These are the
 * elements the engine's pack fragments keep whole and its send positions snap to.  Same return
 * convention as ddt_type_to_opal_desc. */
int64_t ddt_type_to_opal_opt_desc(const ddt_datatype_t *type, void *out, size_t cap, uint32_t *flags);

/* ================= convertor (opal/datatype/opal_convertor.h) ================= */

ddt_convertor_t *ddt_convertor_create(void);                   /* opal_convertor_create */
void ddt_convertor_destroy(ddt_convertor_t *conv);             /* OBJ_RELEASE(convertor) */
/* opal_convertor_prepare_for_send (opal_convertor.c:648-696) */
int ddt_convertor_prepare_for_send(ddt_convertor_t *conv, const ddt_datatype_t *type, size_t count,
                                   const void *buf);
/* opal_convertor_prepare_for_recv (opal_convertor.c:616-646) */
int ddt_convertor_prepare_for_recv(ddt_convertor_t *conv, const ddt_datatype_t *type, size_t count,
                                   void *buf);
/* external32 data representation: MPI_Pack_external / MPI_Unpack_external /
 * MPI_Pack_external_size (ompi_datatype_external.c:33-135 over the external32 convertor
 * of ompi_datatype_external32.c:35-38).  Big-endian elements; MPI_LONG / MPI_UNSIGNED_LONG
 * travel as 4 bytes; long double types are refused (DDT_ERR_NOT_SUPPORTED).  The user
 * buffer must be device memory; the external buffer may be device or host memory.
 * `datarep` is accepted and ignored, as in the reference.  Synchronous. */
int ddt_pack_external_size(const char *datarep, size_t incount, const ddt_datatype_t *type,
                           ptrdiff_t *size);
int ddt_pack_external(const char *datarep, const void *inbuf, size_t incount,
                      const ddt_datatype_t *type, void *outbuf, ptrdiff_t outsize,
                      ptrdiff_t *position);
int ddt_unpack_external(const char *datarep, const void *inbuf, ptrdiff_t insize,
                        ptrdiff_t *position, void *outbuf, size_t outcount,
                        const ddt_datatype_t *type);

/* Raw iovec export: opal_convertor_raw (opal_convertor_raw.c:65-283, prototype
 * opal_convertor.h:352-354).  Fills iov[0..*iov_count) with the user-memory regions of the
 * type map in type-map order from the current position, merging adjacent regions
 * (opal_convertor_merge_iov :41-58); stops before a region that needs one more iovec.
 * *length = bytes described.  Returns 1 when the whole message has been described, else 0.
 * No data moves, so the buffer may be host, device or NULL (the reference's callers prepare
 * on NULL: ddt_raw2.c:45).  ddt_convertor_prepare_for_raw is prepare_for_send without the
 * accelerator check. */
int ddt_convertor_prepare_for_raw(ddt_convertor_t *conv, const ddt_datatype_t *type, size_t count,
                                  const void *buf);
int32_t ddt_convertor_raw(ddt_convertor_t *conv, struct iovec *iov, uint32_t *iov_count,
                          size_t *length);
/* opal_convertor_pack (opal_convertor.c:255-305): fAdvance slot = opal_pack_accelerator_simple
 * (opal_datatype_pack_accelerator.c:161-295).  Never splits a predefined element. */
int32_t ddt_convertor_pack(ddt_convertor_t *conv, struct iovec *iov, uint32_t *out_size,
                           size_t *max_data);
/* opal_convertor_unpack (opal_convertor.c:307-349): fAdvance slot = opal_unpack_accelerator_simple
 * (opal_datatype_unpack_accelerator.c:210-368).  Accepts arbitrary byte windows. */
int32_t ddt_convertor_unpack(ddt_convertor_t *conv, struct iovec *iov, uint32_t *out_size,
                             size_t *max_data);
/* opal_convertor_set_position (opal_convertor.h:357-394).  A send convertor that is not NO_OP
 * (the type has gaps and is not one contiguous instance) lands on the predefined-element
 * boundary at or below *position and returns it there, as opal_convertor_position_generic
 * does (opal_convertor.c:458-470); a receive convertor takes any byte. */
int ddt_convertor_set_position(ddt_convertor_t *conv, size_t *position);
/* The send-side snap alone: the packed position of the predefined-element boundary of the
 * committed type map at or below `position` (opal_datatype_position.c:167-367 followed by
 * bConverted -= partial_length, opal_convertor.c:465-468).  For the fPosition of a bridge. */
int ddt_type_snap_position(const ddt_datatype_t *type, size_t position, size_t *snapped);
/* opal_convertor_get_packed_size / get_unpacked_size (opal_convertor.h:240-262) */
int ddt_convertor_get_packed_size(const ddt_convertor_t *conv, size_t *size);
/* bConverted and CONVERTOR_COMPLETED (opal_convertor.h:137-148) */
int ddt_convertor_get_position(const ddt_convertor_t *conv, size_t *position);
int ddt_convertor_is_completed(const ddt_convertor_t *conv);
/* opal_convertor_clone (opal_convertor.c:708-756) and clone_with_position
 * (opal_convertor.h:399-404): `dst` gets `src`'s type, count, buffer, direction and stream.
 * copy_stack != 0 also copies the position; otherwise the clone starts at position 0 (the
 * reference leaves bConverted = -1 until a set_position).  `dst`'s own staging buffers stay. */
int ddt_convertor_clone(const ddt_convertor_t *src, ddt_convertor_t *dst, int copy_stack);
int ddt_convertor_clone_with_position(const ddt_convertor_t *src, ddt_convertor_t *dst, int copy_stack,
                                      size_t *position);
/* opal_convertor_need_buffers (opal_convertor.h:231-240): 0 when the user buffer itself is the
 * packed stream (no gaps, or one contiguous instance), 1 otherwise; always homogeneous. */
int ddt_convertor_need_buffers(const ddt_convertor_t *conv);
/* opal_convertor_get_current_pointer / get_offset_pointer (opal_convertor.h:300-312):
 * base + position (or offset) + true_lb; meaningful for contiguous types. */
int ddt_convertor_get_current_pointer(const ddt_convertor_t *conv, void **position);
int ddt_convertor_get_offset_pointer(const ddt_convertor_t *conv, size_t offset, void **position);
/* opal_convertor_get_unpacked_size: local size (== packed size, homogeneous). */
int ddt_convertor_get_unpacked_size(const ddt_convertor_t *conv, size_t *size);
/* opal_convertor_cleanup (opal_convertor.h:208-219): back to an unprepared, completed
 * convertor that can be prepared again (freelist reuse); stream and staging are kept. */
int ddt_convertor_cleanup(ddt_convertor_t *conv);
/* CONVERTOR_ACCELERATOR_ASYNC + convertor->stream (opal_convertor.h:150, pml_ob1_recvreq.c:627-663):
 * with async != 0 the kernels are enqueued on `hip_stream` and pack/unpack return without
 * synchronizing; the caller records an event on the stream.  async == 0 (default) = synchronous. */
int ddt_convertor_set_stream(ddt_convertor_t *conv, void *hip_stream, int async);

/* ================= MPI front end (ompi/mpi/c/pack.c.in, unpack.c.in, pack_size.c.in) ================= */

/* MPI_Pack: packs incount instances at inbuf into outbuf[*position ..], advances *position. */
int ddt_pack(const void *inbuf, size_t incount, const ddt_datatype_t *type, void *outbuf,
             size_t outsize, size_t *position);
/* MPI_Unpack */
int ddt_unpack(const void *inbuf, size_t insize, size_t *position, void *outbuf, size_t outcount,
               const ddt_datatype_t *type);
/* MPI_Pack_size (homogeneous: incount * size) */
int ddt_pack_size(size_t incount, const ddt_datatype_t *type, size_t *size);

/* ================= engine extras ================= */

/* Windowed pack/unpack on a stream, UCX generic-datatype form
 * (pml_ucx_datatype.c:72-123): pack [offset, offset+max_len) of the packed stream of
 * `count` instances at `buf`; *len returns the bytes produced. Byte-exact window. */
int ddt_pack_window(const ddt_datatype_t *type, size_t count, const void *buf, size_t offset,
                    void *dst, size_t max_len, size_t *len, void *hip_stream);
int ddt_unpack_window(const ddt_datatype_t *type, size_t count, void *buf, size_t offset,
                      const void *src, size_t len, void *hip_stream);
/* Device typed copy (opal_datatype_copy_content_same_ddt, opal_datatype_copy.c:141-178):
 * copies count instances from src layout to dst layout of the same type, D2D, one launch on
 * `hip_stream`; synchronous like the reference (the data is in place on return). */
int ddt_copy_content_same_ddt(const ddt_datatype_t *type, size_t count, void *dst, const void *src,
                              void *hip_stream);

/* ompi_datatype_sndrcv (ompi/datatype/ompi_datatype_sndrcv.c:46-126): local send/recv between
 * two typed device buffers (collectives' self copies).  A NULL type marks that side as
 * MPI_PACKED (count = bytes).  Same type: one typed-copy launch; two types: pack into HBM
 * scratch and unpack, stream-ordered; synchronous on `hip_stream`.  Truncation rules and the
 * DDT_ERR_TRUNCATE cases are the reference's. */
int ddt_sndrcv(const void *sbuf, size_t scount, const ddt_datatype_t *stype, void *rbuf, size_t rcount,
               const ddt_datatype_t *rtype, void *hip_stream);
/* ompi_datatype_get_elements (ompi/datatype/ompi_datatype_get_elements.c:30-76, MPI_Get_elements):
 * basic elements in the first `ucount` packed bytes of a message of this type; whole instances
 * count every element of the type map, a leftover is counted by opal_datatype_get_element_count's
 * walk (opal_datatype_get_count.c:32-92).  DDT_ERR_VALUE_OUT_OF_BOUNDS when the bytes end inside
 * an element (MPI_UNDEFINED). */
int ddt_get_elements(const ddt_datatype_t *type, size_t ucount, size_t *count);
/* Plan introspection for tests/benchmarks: number of leaves, device metadata bytes. */
int ddt_type_plan_info(const ddt_datatype_t *type, int64_t *out4);
/* Which engine whole-message moves of this type use: out4 = [state, device bytes, chunks,
 * U slots] of the address-ordered index-list engine (ddt_sorted.hip); state 1 = built and in
 * use, 0 = not tried yet (built at the first whole-message pack/unpack), -1 = not applicable
 * (the per-block list kernel runs). */
int ddt_type_engine_info(const ddt_datatype_t *type, int64_t *out4);
/* Descriptor-set cache of a type's plan: out4 = [cached sets, evicted sets waiting for their
 * retirement events, sets held for captured graphs, HIP device of the plan (-1 before first
 * use)].  Sets are keyed by the request's shape and pointer alignment, not by buffer address. */
int ddt_type_cache_info(const ddt_datatype_t *type, int64_t *out4);
/* Device memory of the engine's own metadata (descriptor sets, index lists, address-ordered
 * tables, staging and scratch) is cached, not freed: destroying a datatype never waits for
 * the device nor calls hipFree (which synchronises the whole device and breaks another
 * thread's stream capture).  Its memory is reused once the streams that launched its work
 * pass fence events recorded at destruction; memory a captured graph may read is kept.
 * ddt_trim (torch.cuda.empty_cache's analogue) synchronises the device and returns every
 * cached block to HIP.  ddt_pool_info: out6 = [free blocks, free bytes, fenced blocks, fenced
 * bytes, blocks kept for graphs, blocks in use]. */
int ddt_trim(void);
int ddt_pool_info(int64_t *out6);
/* Argument-free launches: a descriptor set launched on the same buffers again within its last 8 launches
 * (up to 8 bindings per set) is bound to one of 32 launch records per direction in device memory, and its later launches on
 * those buffers take no kernel arguments (HIP writes device-resident kernel arguments across
 * PCIe: ~2.9 us of host time per launch with arguments, 0.7 us without).  ddt_slot_info: out4 =
 * [pack slots bound, unpack slots bound (current device), binds so far, argument-free launches
 * so far].  ddt_tune("slots", 0) turns them off; ddt_trim ends every binding. */
int ddt_slot_info(int64_t *out4);
/* Diagnostic: the state of launch slot k of direction dir (0 pack, 1 unpack) on the current
 * device: bit 0 bound, bit 1 ending (its binding ended but the fences on its streams could not be
 * recorded yet, e.g. one is capturing: never rebound before they are), bits 8.. the number of
 * streams its binding launched on; -1 when no slot of that direction exists yet. */
int ddt_slot_state(int dir, int k);
/* Synchronous completion (round 6): a synchronous pack / unpack (MPI_Pack, MPI_Unpack, a
 * convertor without the async flag) returns once a signal kernel enqueued behind its work has
 * written a pinned host word, instead of HIP's ~9.5 us completion round trip; it falls back to
 * hipStreamSynchronize when the stream captures, all 16 signal slots are taken, a window is in
 * host memory, or the word is not seen within 20 ms.  ddt_tune("sigsync", 0) turns it off.
 * out3 = [calls completed by the signal, signal fallbacks (timeout), plain stream syncs]. */
int ddt_sync_info(int64_t *out3);
/* ---- introspection for the CPU test-suite (no data movement; never used by pack/unpack) ----
 * ddt_type_plan_leaves: serialises the plan's leaf streams as int64 records
 *   [kind, blen, src_off, dst_off, ndim, list_leaf_index, (cnt, sstr, dstr) x ndim] and returns
 *   the number of int64 written (or the number needed when cap is too small, as a negative).
 * ddt_debug_items: the launch descriptors (ddt_device.h Item, raw bytes) that pack/unpack would
 *   run for the packed window [w0, w1) of `count` instances at `user` with the packed pointer
 *   `pk` holding byte w0; *nitems receives the count, *item_size the size of one Item.
 * ddt_type_plan_list: host copy of index-list leaf `leaf`: block displacements and lengths.
 * ddt_debug_host_window: 1 (and the device address) when a host iovec [p, p + n) would be moved
 *   by the kernel itself over PCIe (inside one pinned allocation or registration), else 0: the
 *   iovec goes through HBM staging. */
int64_t ddt_type_plan_leaves(const ddt_datatype_t *type, int64_t *out, size_t cap);
int ddt_debug_items(const ddt_datatype_t *type, size_t count, uint64_t user, uint64_t pk,
                    uint64_t w0, uint64_t w1, int same_layout, void *out, size_t cap_bytes,
                    size_t *nitems, size_t *item_size);
int64_t ddt_type_plan_list(const ddt_datatype_t *type, size_t leaf, int64_t *disp, uint64_t *len,
                           size_t cap);
int ddt_debug_host_window(const void *p, size_t n, uint64_t *device_addr);
/* Tuning knobs for A/B measurements (affect descriptor sets built afterwards):
 * "nt" = user-side non-temporal gathers (-1 auto = off since round 3, 0 off, 1 on); "task_kb" = packed KiB per
 * workgroup (0 adaptive); "policy" = task sizing (0 v0, 1 per-leaf passes); "interleave" =
 * reorder a pack's items in runs of this many tasks (0 off, default); "uinterleave" = the same for
 * an unpack (256 default, -1 as "interleave"); "wt" = write-through stores (-1 auto,
 * 0 off, 1 every sparse leaf, 2 all); "sorted" = address-ordered list engine (-1 auto from
 * 1 Mi blocks, 0 off, n > 0 from n blocks; read when a type's plan first runs);
 * "spol" = the address-ordered engine's
 * access-policy bits (ddt_sorted.hip POL_*); "ptr" = launch reused descriptor sets by pointer
 * (1, default) or always from the kernel-argument segment (0); "xcd" = mapping of workgroups to
 * tasks (-1, default: each XCD runs a contiguous slab of a streaming or line-dense leaf, sparse
 * gathers stay round-robin; 0: all round-robin; 1: all slabs); "xchunk" = tasks per XCD run for
 * slab items (0, default: one slab per XCD); "snt" = cache policy of streaming leaves (-1 auto:
 * non-temporal loads, and stores too in a launch with isolated narrow blocks; -3 loads only; else
 * an Item::nt mode 0-5); "spass" = workgroup passes per streaming task; "stask" = bytes per
 * streaming task (0, default: spass passes); "dense" = line-dense records moved through LDS
 * with whole-line accesses (-1 auto, 0 off, n chunks per task); "dsplit" = such an unpack runs
 * each task as two workgroups (1 default, 0 off); "dfast" = a large single-item line-dense launch
 * passes its fields by value, one workgroup per chunk (bit 0 pack, default; bit 1 unpack); "hostdirect" =
 * pinned host iovecs moved by the kernel over PCIe (bit 0 unpack, bit 1 pack; 3 default, 0 =
 * HBM staging); "hd_grid" / "hd_grid_pack" = workgroup cap of such an unpack / pack launch (256 / 0 default,
 * 0 none); "stage_mb" =
 * staging buffer MiB for pageable host iovecs (256 default; read when a convertor first stages); "sseg" =
 * address-ordered engine segment bytes (32, 64 default, 128); "sunroll" = its pack-1 elements per
 * thread in flight (4, 8, 16 default); "s2unroll" = the same for its unpack pass 2' (4, 8
 * default, 16);
 * "reset" = restore the defaults.
 * Environment: DDT_NT, DDT_TASK_KB, DDT_WT, DDT_XCD. */
int ddt_tune(const char *key, long value);
/* Library self-check of host-side index arithmetic (fast division); returns 0 on success. */
int ddt_selftest(void);
const char *ddt_version(void);
/* sha256 of the sources the library was linked from (scripts/srcsha.py; build provenance). */
const char *ddt_build_id(void);
/* Message of the last failing call on this thread (empty if none). */
const char *ddt_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* DDT_HIP_H */
