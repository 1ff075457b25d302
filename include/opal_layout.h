/*
 * opal_layout.h -- the in-memory layout of the Open MPI objects the fAdvance bridge reads
 * and writes, restated for an LP64 build with OPAL_ENABLE_DEBUG = 0 and
 * OPAL_MAX_OBJECT_NAME = 64 (the configuration SURVEY.md Appendix B builds).
 *
 * Inside an Open MPI build tree the bridge includes the real headers instead
 * ("opal/datatype/opal_convertor.h", "opal/datatype/opal_datatype_internal.h"); this file
 * exists so the bridge compiles and is tested here without Open MPI's configure step.
 * The _Static_asserts pin every offset the bridge touches to the layout notes of the
 * reference headers, so a drift between the two is a compile error, not a silent misread.
 *
 *   opal_object_t      opal/class/opal_object.h:189-202
 *   opal_datatype_t    opal/datatype/opal_datatype.h:162-212 (200 bytes, note at :204-211)
 *   dt_elem_desc_t     opal/datatype/opal_datatype_internal.h:119-169 (32-byte union)
 *   dt_stack_t         opal/datatype/opal_convertor.h:111-117
 *   opal_convertor_t   opal/datatype/opal_convertor.h:125-170 (cache lines at :136, :149)
 *   flags              opal/datatype/opal_convertor.h:55-76, opal_datatype.h:79-142
 *   stream             opal/mca/accelerator/accelerator.h:114-123
 *   return codes       opal/include/opal/constants.h:29-48
 */
#ifndef OPAL_LAYOUT_H
#define OPAL_LAYOUT_H

#include <stddef.h>
#include <stdint.h>
#include <sys/uio.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- return codes ---- */
#define OPAL_SUCCESS 0
#define OPAL_ERROR (-1)
#define OPAL_ERR_OUT_OF_RESOURCE (-2)
#define OPAL_ERR_BAD_PARAM (-5)
#define OPAL_ERR_NOT_SUPPORTED (-8)

/* ---- datatype flags (opal_datatype.h:79-142) ---- */
#define OPAL_DATATYPE_FLAG_PREDEFINED 0x0002u
#define OPAL_DATATYPE_FLAG_COMMITTED 0x0004u
#define OPAL_DATATYPE_FLAG_OVERLAP 0x0008u
#define OPAL_DATATYPE_FLAG_CONTIGUOUS 0x0010u
#define OPAL_DATATYPE_FLAG_NO_GAPS 0x0020u
#define OPAL_DATATYPE_FLAG_DATA 0x0100u
#define OPAL_DATATYPE_OPTIMIZED_RESTRICTED 0x00010000u

/* ---- descriptor entry type ids (opal_datatype_internal.h:71-100) ---- */
#define OPAL_DATATYPE_LOOP 0
#define OPAL_DATATYPE_END_LOOP 1

/* ---- convertor flags (opal_convertor.h:55-76) ---- */
#define CONVERTOR_DATATYPE_MASK 0x0000FFFFu
#define CONVERTOR_UNSAFE_SPLIT 0x00100000u
#define CONVERTOR_SEND_CONVERSION 0x00200000u
#define CONVERTOR_RECV 0x00400000u
#define CONVERTOR_SEND 0x00800000u
#define CONVERTOR_HOMOGENEOUS 0x01000000u
#define CONVERTOR_NO_OP 0x02000000u
#define CONVERTOR_COMPLETED 0x04000000u
#define CONVERTOR_HAS_REMOTE_SIZE 0x08000000u
#define CONVERTOR_ACCELERATOR 0x10000000u
#define CONVERTOR_ACCELERATOR_ASYNC 0x20000000u
#define CONVERTOR_ACCELERATOR_UNIFIED 0x40000000u

typedef struct opal_object_t {
    void *obj_class;                  /* opal_class_t * */
    volatile int32_t obj_reference_count;
} opal_object_t;

/* ---- the committed description: 32-byte entries ---- */
typedef struct ddt_elem_id_description {
    uint16_t flags;
    uint16_t type;
} ddt_elem_id_description;

typedef struct ddt_elem_desc {    /* DATA: count blocks of blocklen elements at stride extent */
    ddt_elem_id_description common;
    uint32_t count;
    size_t blocklen;
    ptrdiff_t extent;
    ptrdiff_t disp;
} ddt_elem_desc_t;

typedef struct ddt_loop_desc {    /* LOOP: loops iterations of the next items-1 entries */
    ddt_elem_id_description common;
    uint32_t items;
    uint32_t loops;
    size_t unused;
    ptrdiff_t extent;
} ddt_loop_desc_t;

typedef struct ddt_endloop_desc { /* END_LOOP: closes the loop `items` entries back */
    ddt_elem_id_description common;
    uint32_t items;
    uint32_t unused;
    size_t size;
    ptrdiff_t first_elem_disp;
} ddt_endloop_desc_t;

typedef union dt_elem_desc {
    ddt_elem_desc_t elem;
    ddt_loop_desc_t loop;
    ddt_endloop_desc_t end_loop;
} dt_elem_desc_t;

typedef struct dt_type_desc_t {
    size_t length;                    /* opal_datatype_count_t */
    size_t used;
    dt_elem_desc_t *desc;
} dt_type_desc_t;

typedef struct opal_datatype_t {
    opal_object_t super;
    uint32_t flags;
    uint32_t bdt_used;
    size_t size;
    ptrdiff_t true_lb;
    ptrdiff_t true_ub;
    ptrdiff_t lb;
    ptrdiff_t ub;
    size_t nbElems;
    uint16_t id;
    uint16_t align;
    uint32_t stack_depth;
    char name[64];
    dt_type_desc_t desc;
    dt_type_desc_t opt_desc;
    size_t *ptypes;
} opal_datatype_t;

/* ---- convertor ---- */
typedef struct dt_stack_t {
    int32_t index;
    int16_t type;
    int16_t padding;
    size_t count;
    ptrdiff_t disp;
} dt_stack_t;

typedef struct opal_accelerator_stream_t {
    opal_object_t super;
    void *stream;                     /* rocm component: a malloc'ed hipStream_t cell, i.e. a
                                         hipStream_t * (accelerator_rocm_module.c:80,176-182) */
} opal_accelerator_stream_t;
/* MCA_ACCELERATOR_STREAM_DEFAULT (accelerator.h:123): the default stream, not an object */
#define OPAL_ACCELERATOR_STREAM_DEFAULT ((opal_accelerator_stream_t *) 0x00000002)

typedef struct opal_convertor_t opal_convertor_t;
typedef int32_t (*convertor_advance_fct_t)(opal_convertor_t *pConvertor, struct iovec *iov,
                                           uint32_t *out_size, size_t *max_data);
typedef int32_t (*convertor_position_fct_t)(opal_convertor_t *pConvertor, size_t *position);
typedef void *(*memcpy_fct_t)(void *dest, const void *src, size_t n, opal_convertor_t *pConvertor);

#define DT_STATIC_STACK_SIZE 5

struct opal_convertor_t {
    opal_object_t super;
    const opal_datatype_t *pDesc;
    const dt_type_desc_t *use_desc;
    size_t count;                     /* opal_datatype_count_t */
    size_t remote_size;
    void *master;                     /* struct opal_convertor_master_t * */
    convertor_advance_fct_t fAdvance;
    /* cache line 1 */
    size_t bConverted;
    size_t partial_length;
    size_t local_size;
    unsigned char *pBaseBuf;
    dt_stack_t *pStack;
    memcpy_fct_t cbmemcpy;
    uint32_t flags;
    uint32_t stack_pos;
    uint32_t stack_size;
    uint32_t remoteArch;
    /* cache line 2 */
    const size_t *sizes;
    convertor_position_fct_t fPosition;
    dt_stack_t static_stack[DT_STATIC_STACK_SIZE];
    opal_accelerator_stream_t *stream;
};

#ifndef __cplusplus
_Static_assert(sizeof(dt_elem_desc_t) == 32, "dt_elem_desc_t is 32 bytes");
_Static_assert(offsetof(ddt_elem_desc_t, blocklen) == 8 && offsetof(ddt_elem_desc_t, disp) == 24,
               "DATA entry layout");
_Static_assert(offsetof(ddt_loop_desc_t, loops) == 8 && offsetof(ddt_loop_desc_t, extent) == 24,
               "LOOP entry layout");
_Static_assert(offsetof(ddt_endloop_desc_t, size) == 16, "END_LOOP entry layout");
_Static_assert(sizeof(opal_datatype_t) == 200, "opal_datatype.h:204-211: 200 bytes in LP64");
_Static_assert(offsetof(opal_datatype_t, opt_desc) == 168, "opt_desc offset");
_Static_assert(offsetof(opal_convertor_t, bConverted) == 64, "opal_convertor.h:136 cache line");
_Static_assert(offsetof(opal_convertor_t, sizes) == 128, "opal_convertor.h:149 cache line");
_Static_assert(sizeof(dt_stack_t) == 24, "dt_stack_t layout");
_Static_assert(offsetof(opal_convertor_t, stream) == 264, "stream offset");
#endif

#ifdef __cplusplus
}
#endif
#endif /* OPAL_LAYOUT_H */
