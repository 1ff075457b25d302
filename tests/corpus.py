"""The reference's datatype corpus (ompi/test/datatype/datatype_corpus.c) restated as
recipes plus independent by-hand packers.

Each entry: (name, recipe, byhand) where byhand(count) returns the list of
(offset, length) regions the reference's pack_byhand_* copies, in order, relative to
the buffer pointer handed to MPI_Pack (opt_desc_equiv.c:330-381: the same `src` goes to
both).  These by-hand baselines are the reference's own known answers for the packed
stream; they pin the oracle (tests/test_cpu_golden.py) and, through it, the HIP engine.
Constants and offsets follow datatype_corpus.c line for line (cited per entry).
"""
from __future__ import annotations

DOUBLE, LONG, CHAR, INT, FLOAT = 16, 25, 4, 6, 15

# datatype_corpus.c:314-355 (enum of DDTBench sizes)
STEP = 37
FFT_DIM, FFT_PROCS = 256, 2
MILC = 8
NAS_LU_DIM2 = NAS_LU_DIM3 = 12
NAS_LU_X_DIM2, NAS_LU_CELL = 1020, 5
MG1, MG2, MG3 = 34, 18, 18
LAMMPS_FULL_DIM, LAMMPS_FULL_ICOUNT = 3534, 3062
LAMMPS_ATOMIC_DIM, LAMMPS_ATOMIC_ICOUNT = 4084, 243
SPEC_OC_DIM, SPEC_OC_ICOUNT = 3697, 493
SPEC_CM_DIM_CM, SPEC_CM_DIM_IC, SPEC_CM_ICOUNT_CM, SPEC_CM_ICOUNT_IC = 39929, 1225, 1957, 245
SPEC_MT = (3, 2, 6200)
WRF_N2, WRF_N3, WRF_N4 = 4, 3, 2
WRF_D1, WRF_D2, WRF_D3 = 19, 65, 24
WRF_LIMIT4, WRF_IS, WRF_KS, WRF_JS, WRF_FIRST = 2, 9, 0, 4, 1
WRF_S1, WRF_S2, WRF_S3 = 3, 65, 16


def ddt_index(i, dim):   # datatype_corpus.c:480-483
    return (i * STEP) % dim


def B(t):
    return ("basic", t)


# ---------------------------------------------------------------- shapes
def merged_contig_with_gaps():
    """:59-97 struct{double,long,char} resized to sizeof (24); by-hand :1045-1055."""
    rec = ("resized", ("struct", [1, 1, 1], [0, 8, 16], [B(DOUBLE), B(LONG), B(CHAR)]), 0, 24)

    def byhand(count):
        return [(i * 24, 17) for i in range(count)]
    return rec, byhand


def struct_constant_gap_resized():
    """:99-123 struct{double@8,long@16} resized to 24; by-hand :1069-1081."""
    rec = ("resized", ("struct", [1, 1], [8, 16], [B(DOUBLE), B(LONG)]), 0, 24)
    return rec, lambda count: [(i * 24 + 8, 16) for i in range(count)]


def _const_gap_byhand(count):
    """:1098-1113: 80 blocks of 100 doubles at a 101-double stride."""
    ext = 79 * 101 * 8 + 100 * 8
    return [(i * ext + b * 101 * 8, 800) for i in range(count) for b in range(80)]


def indexed_constant_gap():
    """:126-161 struct of 80 x (100 doubles) at 101-double steps (create_struct path)."""
    dbl = B(DOUBLE)
    rec = ("struct", [100] * 80, [i * 8 * 101 for i in range(80)], [dbl] * 80)
    return rec, _const_gap_byhand


def struct_constant_gap():
    """:163-196 the same layout through a struct-derived payload subtype."""
    payload = ("struct", [100], [0], [B(DOUBLE)])
    rec = ("struct", [1] * 80, [i * 8 * 101 for i in range(80)], [payload] * 80)
    return rec, _const_gap_byhand


def optimized_indexed_constant_gap():
    """:198-208 vector(80, 100, 101, double)."""
    return ("vector", 80, 100, 101, B(DOUBLE)), _const_gap_byhand


# ddt_gap layout (:215-219): {int v1; int gap1; internal_struct{int i[2]; float f;} is[3];}
# sizeof(internal_struct) = 12, offsetof(is) = 8, sizeof(ddt_gap) = 44
def _indexed_gap_byhand(count):
    """:1164-1187"""
    rec_ext, payload_off, payload_len, lead = 44, 8, 36, 4
    ext = 10 * rec_ext
    out = []
    for i in range(count):
        base = i * ext
        out.append((base, lead))
        for r in range(9):
            out.append((base + r * rec_ext + payload_off, payload_len + lead))
        out.append((base + 9 * rec_ext + payload_off, payload_len))
    return out


def indexed_gap():
    """:221-259 contiguous(10, struct{int, contiguous(3, struct{int[2], float})})."""
    dt1 = ("struct", [2, 1], [0, 8], [B(INT), B(FLOAT)])
    dt2 = ("contig", 3, dt1)
    dt3 = ("struct", [1, 1], [0, 8], [B(INT), dt2])
    return ("contig", 10, dt3), _indexed_gap_byhand


def indexed_gap_optimized():
    """:261-302 the hand-built optimizer target, resized to 440."""
    dt2 = ("resized", ("contig", 10, B(FLOAT)), 0, 44)
    st = ("struct", [1, 9, 9], [0, 8, 44 * 9 + 8], [B(FLOAT), dt2, B(FLOAT)])
    return ("resized", st, 0, 440), _indexed_gap_byhand


def fft2d_scatter():
    """:513-529; by-hand :1233-1253"""
    cols = FFT_DIM // FFT_PROCS
    cplx = ("contig", 2, B(DOUBLE))
    vec = ("vector", cols, 1, FFT_DIM, cplx)
    rec = ("contig", cols, ("resized", vec, 0, 16))

    def byhand(count):
        ext = cols * 16
        return [(d * ext + (c + r * FFT_DIM) * 16, 16) for d in range(count)
                for c in range(cols) for r in range(cols)]
    return rec, byhand


def fft2d_gather():
    """:531-545; by-hand :1277-1294"""
    cols = FFT_DIM // FFT_PROCS
    cplx = ("contig", 2, B(DOUBLE))
    rec = ("resized", ("vector", cols, cols, FFT_DIM, cplx), 0, cols * 16)

    def byhand(count):
        return [(d * cols * 16 + r * FFT_DIM * 16, cols * 16) for d in range(count) for r in range(cols)]
    return rec, byhand


def milc_su3_zdown():
    """:547-566; by-hand :1315-1341"""
    su3 = ("contig", 6, B(FLOAT))
    tmp = ("vector", MILC, MILC * MILC // 2, MILC * MILC * MILC // 2, su3)
    stride = 24 * MILC * MILC * MILC * MILC // 2
    rec = ("hvector", 2, 1, stride, tmp)

    def byhand(count):
        block = (MILC * MILC // 2) * 24
        tstride = (MILC * MILC * MILC // 2) * 24
        textent = (MILC - 1) * tstride + block
        ext = stride + textent
        return [(d * ext + z * stride + t * tstride, block) for d in range(count)
                for z in range(2) for t in range(MILC)]
    return rec, byhand


def nas_lu_y():
    """:568-578; by-hand :1371-1386"""
    rec = ("vector", NAS_LU_DIM3, 1, NAS_LU_DIM2 + 2, ("contig", NAS_LU_CELL, B(DOUBLE)))

    def byhand(count):
        blk = NAS_LU_CELL * 8
        st = (NAS_LU_DIM2 + 2) * blk
        ext = (NAS_LU_DIM3 - 1) * st + blk
        return [(d * ext + r * st, blk) for d in range(count) for r in range(NAS_LU_DIM3)]
    return rec, byhand


def nas_lu_x():
    """:580-588; by-hand :1405-1411"""
    n = NAS_LU_CELL * NAS_LU_X_DIM2 * 8
    return ("contig", NAS_LU_CELL * NAS_LU_X_DIM2, B(DOUBLE)), lambda count: [(0, n * count)]


def nas_mg_x():
    """:590-603; by-hand :1421-1440"""
    zs = MG1 * MG2 * 8
    rec = ("hvector", MG3 - 2, 1, zs, ("vector", MG2 - 2, 1, MG1, B(DOUBLE)))

    def byhand(count):
        ys = MG1 * 8
        ext = (MG3 - 3) * zs + (MG2 - 3) * ys + 8
        return [(d * ext + z * zs + y * ys, 8) for d in range(count)
                for z in range(MG3 - 2) for y in range(MG2 - 2)]
    return rec, byhand


def nas_mg_y():
    """:605-614; by-hand :1463-1478"""
    rec = ("vector", MG3 - 2, MG1 - 2, MG1 * MG2, B(DOUBLE))

    def byhand(count):
        row = (MG1 - 2) * 8
        zs = MG1 * MG2 * 8
        ext = (MG3 - 3) * zs + row
        return [(d * ext + z * zs, row) for d in range(count) for z in range(MG3 - 2)]
    return rec, byhand


def nas_mg_z():
    """:616-624; by-hand :1497-1512"""
    rec = ("vector", MG2 - 2, MG1 - 2, MG1, B(DOUBLE))

    def byhand(count):
        row = (MG1 - 2) * 8
        ys = MG1 * 8
        ext = (MG2 - 3) * ys + row
        return [(d * ext + y * ys, row) for d in range(count) for y in range(MG2 - 2)]
    return rec, byhand


def lammps_full():
    """:626-676 send type; by-hand :1531-1562"""
    D, N = LAMMPS_FULL_DIM, LAMMPS_FULL_ICOUNT
    i1 = ("indexed_block", 1, [ddt_index(i, D) for i in range(N)], B(DOUBLE))
    i3 = ("indexed_block", 3, [3 * ddt_index(i, D) for i in range(N)], B(DOUBLE))
    offs = [0] + [3 * D * 8 + k * D * 8 for k in range(5)]
    ext = offs[-1] + D * 8
    rec = ("resized", ("struct", [1] * 6, offs, [i3] + [i1] * 5), 0, ext)

    def byhand(count):
        out = []
        for d in range(count):
            base = d * ext
            out += [(base + 3 * ddt_index(i, D) * 8, 24) for i in range(N)]
            for f in range(5):
                out += [(base + offs[1 + f] + ddt_index(i, D) * 8, 8) for i in range(N)]
        return out
    return rec, byhand


def lammps_atomic():
    """:678-726 send type; by-hand :1593-1622"""
    D, N = LAMMPS_ATOMIC_DIM, LAMMPS_ATOMIC_ICOUNT
    i1 = ("indexed_block", 1, [ddt_index(i, D) for i in range(N)], B(DOUBLE))
    i3 = ("indexed_block", 3, [3 * ddt_index(i, D) for i in range(N)], B(DOUBLE))
    offs = [0] + [3 * D * 8 + k * D * 8 for k in range(3)]
    ext = offs[-1] + D * 8
    rec = ("resized", ("struct", [1] * 4, offs, [i3] + [i1] * 3), 0, ext)

    def byhand(count):
        out = []
        for d in range(count):
            base = d * ext
            out += [(base + 3 * ddt_index(i, D) * 8, 24) for i in range(N)]
            for f in range(3):
                out += [(base + offs[1 + f] + ddt_index(i, D) * 8, 8) for i in range(N)]
        return out
    return rec, byhand


def specfem3d_oc():
    """:728-741; by-hand :1651-1667"""
    rec = ("resized", ("indexed_block", 1, [ddt_index(i, SPEC_OC_DIM) for i in range(SPEC_OC_ICOUNT)],
                       B(FLOAT)), 0, SPEC_OC_DIM * 4)

    def byhand(count):
        return [(d * SPEC_OC_DIM * 4 + ddt_index(i, SPEC_OC_DIM) * 4, 4) for d in range(count)
                for i in range(SPEC_OC_ICOUNT)]
    return rec, byhand


def specfem3d_cm():
    """:743-774; by-hand :1687-1712"""
    cm = ("indexed_block", 3, [3 * ddt_index(i, SPEC_CM_DIM_CM) for i in range(SPEC_CM_ICOUNT_CM)], B(FLOAT))
    ic = ("indexed_block", 3, [3 * ddt_index(i, SPEC_CM_DIM_IC) for i in range(SPEC_CM_ICOUNT_IC)], B(FLOAT))
    ic_off = 3 * SPEC_CM_DIM_CM * 4
    ext = ic_off + 3 * SPEC_CM_DIM_IC * 4
    rec = ("resized", ("struct", [1, 1], [0, ic_off], [cm, ic]), 0, ext)

    def byhand(count):
        out = []
        for d in range(count):
            base = d * ext
            out += [(base + 3 * ddt_index(i, SPEC_CM_DIM_CM) * 4, 12) for i in range(SPEC_CM_ICOUNT_CM)]
            out += [(base + ic_off + 3 * ddt_index(i, SPEC_CM_DIM_IC) * 4, 12) for i in range(SPEC_CM_ICOUNT_IC)]
        return out
    return rec, byhand


def specfem3d_mt():
    """:776-789 send type vector(6200, 1, 2, contiguous(3 float)); by-hand :1743-1758"""
    d1, d2, d3 = SPEC_MT
    rec = ("vector", d3, 1, d2, ("contig", d1, B(FLOAT)))

    def byhand(count):
        blk = d1 * 4
        st = d2 * blk
        ext = (d3 - 1) * st + blk
        return [(c * ext + i * st, blk) for c in range(count) for i in range(d3)]
    return rec, byhand


def _wrf_offsets():
    a2 = WRF_D1 * WRF_D3
    a3 = WRF_D1 * WRF_D2 * WRF_D3
    a4 = a3 * WRF_LIMIT4
    off3 = WRF_N2 * a2 * 4
    off4 = off3 + WRF_N3 * a3 * 4
    ext = off4 + WRF_N4 * a4 * 4
    return a2, a3, a4, off3, off4, ext


def _wrf_byhand(count):
    """:1774-1838"""
    a2, a3, a4, off3, off4, ext = _wrf_offsets()
    row = WRF_S1 * 4
    out = []
    idx2 = lambda x, y: x + y * WRF_D1  # noqa: E731
    idx3 = lambda x, y, z: x + WRF_D1 * (y + WRF_D2 * z)  # noqa: E731
    idx4 = lambda x, y, z, t: x + WRF_D1 * (y + WRF_D2 * (z + WRF_D3 * t))  # noqa: E731
    for d in range(count):
        base = d * ext
        for a in range(WRF_N2):
            out += [(base + a * a2 * 4 + idx2(WRF_IS, WRF_JS + z) * 4, row) for z in range(WRF_S3)]
        for a in range(WRF_N3):
            ao = off3 + a * a3 * 4
            out += [(base + ao + idx3(WRF_IS, WRF_KS + y, WRF_JS + z) * 4, row)
                    for z in range(WRF_S3) for y in range(WRF_S2)]
        for a in range(WRF_N4):
            ao = off4 + a * a4 * 4
            out += [(base + ao + idx4(WRF_IS, WRF_KS + y, WRF_JS + z, t) * 4, row)
                    for t in range(WRF_FIRST, WRF_LIMIT4) for z in range(WRF_S3) for y in range(WRF_S2)]
    return out


def wrf_vec():
    """:791-867"""
    a2, a3, a4, off3, off4, ext = _wrf_offsets()
    t2 = ("vector", WRF_S3, WRF_S1, WRF_D1, B(FLOAT))
    tmp = ("vector", WRF_S2, WRF_S1, WRF_D1, B(FLOAT))
    stride = WRF_D1 * WRF_D2 * 4
    t3 = ("hvector", WRF_S3, 1, stride, tmp)
    types, disps = [], []
    for i in range(WRF_N2):
        disps.append(i * a2 * 4 + (WRF_IS + WRF_JS * WRF_D1) * 4)
        types.append(t2)
    for i in range(WRF_N3):
        disps.append(off3 + i * a3 * 4 + (WRF_IS + WRF_D1 * (WRF_KS + WRF_D2 * WRF_JS)) * 4)
        types.append(t3)
    stride4 = stride * WRF_D3
    for i in range(WRF_N4):
        t4 = ("hvector", WRF_LIMIT4 - WRF_FIRST, 1, stride4, t3)
        disps.append(off4 + i * a4 * 4
                     + (WRF_IS + WRF_D1 * (WRF_KS + WRF_D2 * (WRF_JS + WRF_D3 * WRF_FIRST))) * 4)
        types.append(t4)
    rec = ("resized", ("struct", [1] * len(types), disps, types), 0, ext)
    return rec, _wrf_byhand


def wrf_subarray():
    """:869-958"""
    a2, a3, a4, off3, off4, ext = _wrf_offsets()
    t2 = ("subarray", [WRF_D3, WRF_D1], [WRF_S3, WRF_S1], [WRF_JS, WRF_IS], 0, B(FLOAT))
    t3 = ("subarray", [WRF_D3, WRF_D2, WRF_D1], [WRF_S3, WRF_S2, WRF_S1], [WRF_JS, WRF_KS, WRF_IS], 0, B(FLOAT))
    t4 = ("subarray", [WRF_LIMIT4, WRF_D3, WRF_D2, WRF_D1],
          [WRF_LIMIT4 - WRF_FIRST, WRF_S3, WRF_S2, WRF_S1], [WRF_FIRST, WRF_JS, WRF_KS, WRF_IS], 0, B(FLOAT))
    types = [t2] * WRF_N2 + [t3] * WRF_N3 + [t4] * WRF_N4
    disps = ([i * a2 * 4 for i in range(WRF_N2)] + [off3 + i * a3 * 4 for i in range(WRF_N3)]
             + [off4 + i * a4 * 4 for i in range(WRF_N4)])
    rec = ("resized", ("struct", [1] * len(types), disps, types), 0, ext)
    return rec, _wrf_byhand


def complex_hvector():
    """:971-1001 hvector(2048, 3, 3*8+4, contiguous(2 float)); by-hand :985-1001"""
    rec = ("hvector", 2048, 3, 28, ("contig", 2, B(FLOAT)))

    def byhand(count):
        ext = 2047 * 28 + 24
        return [(c * ext + b * 28, 24) for c in range(count) for b in range(2048)]
    return rec, byhand


def adv_single_iter_gap():
    """:1943-1964"""
    return (("resized", ("contig", 3, B(INT)), 0, 24),
            lambda count: [(i * 24, 12) for i in range(count)])


def adv_zero_extent_overlap():
    """:1980-1996 (extent 0: every instance is instance zero)"""
    return (("resized", ("contig", 2, B(INT)), 0, 0), lambda count: [(0, 8) for _ in range(count)])


def adv_neg_extent():
    """:2019-2035"""
    return (("resized", ("contig", 2, B(INT)), 0, -8), lambda count: [(-8 * i, 8) for i in range(count)])


def adv_mixed_promote():
    """:2056-2076"""
    pair = ("struct", [1, 1], [0, 4], [B(INT), B(FLOAT)])
    return ("contig", 4, ("resized", pair, 0, 8)), lambda count: [(0, 32 * count)]


def contig():
    """:2125-2128 (MPI_INT as-is); by-hand :1035-1038"""
    return B(INT), lambda count: [(0, 4 * count)]


# The receive types of the three PAIR entries (datatype_corpus.c:626-789): the same packed stream
# into dense storage (lammps: a struct of contiguous runs at the send type's field offsets;
# specfem3d_mt: one contiguous run of floats).
def _lammps_recv(D, N, nfields):
    offs = [0] + [3 * D * 8 + k * D * 8 for k in range(nfields - 1)]
    ext = offs[-1] + D * 8
    types = [("contig", 3 * N, B(DOUBLE))] + [("contig", N, B(DOUBLE))] * (nfields - 1)
    return ("resized", ("struct", [1] * nfields, offs, types), 0, ext)


PAIR_RECV = {
    "ddtbench_lammps_full": _lammps_recv(LAMMPS_FULL_DIM, LAMMPS_FULL_ICOUNT, 6),        # :662-672
    "ddtbench_lammps_atomic": _lammps_recv(LAMMPS_ATOMIC_DIM, LAMMPS_ATOMIC_ICOUNT, 4),  # :712-722
    "ddtbench_specfem3d_mt": ("contig", SPEC_MT[2] * SPEC_MT[0], B(FLOAT)),              # :786-788
}


CORPUS = {
    "contig": contig,
    "indexed_gap": indexed_gap,
    "optimized_indexed_gap": indexed_gap_optimized,
    "constant_gap": indexed_constant_gap,
    "optimized_constant_gap": optimized_indexed_constant_gap,
    "struct_constant_gap": struct_constant_gap,
    "struct_constant_gap_resized": struct_constant_gap_resized,
    "struct_merged_with_gap_resized": merged_contig_with_gaps,
    "ddtbench_fft2d_scatter": fft2d_scatter,
    "ddtbench_fft2d_gather": fft2d_gather,
    "ddtbench_milc_su3_zdown": milc_su3_zdown,
    "ddtbench_nas_lu_y": nas_lu_y,
    "ddtbench_nas_lu_x": nas_lu_x,
    "ddtbench_nas_mg_x": nas_mg_x,
    "ddtbench_nas_mg_y": nas_mg_y,
    "ddtbench_nas_mg_z": nas_mg_z,
    "ddtbench_lammps_full": lammps_full,
    "ddtbench_lammps_atomic": lammps_atomic,
    "ddtbench_specfem3d_oc": specfem3d_oc,
    "ddtbench_specfem3d_cm": specfem3d_cm,
    "ddtbench_specfem3d_mt": specfem3d_mt,
    "ddtbench_wrf_vec": wrf_vec,
    "ddtbench_wrf_subarray": wrf_subarray,
    "complex_hvector": complex_hvector,
    "adv_single_iter_gap": adv_single_iter_gap,
    "adv_zero_extent_overlap": adv_zero_extent_overlap,
    "adv_neg_extent": adv_neg_extent,
    "adv_mixed_promote": adv_mixed_promote,
}
