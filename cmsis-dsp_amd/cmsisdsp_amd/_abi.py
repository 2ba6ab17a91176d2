"""ctypes mirror of include/arm_math.h (struct layouts + prototypes).

The same declarations bind three libraries with the identical C ABI:
  * libcmsisdsp_mi355x.so  — this backend (the product);
  * oracle/_ref/libcmsisdsp_ref.so — the reference scalar C path (test infrastructure);
  * oracle/_build/liboracle.so — the CPU restatement (test infrastructure, `oracle_` prefix).
"""
import ctypes as C

c_f32p = C.POINTER(C.c_float)
c_i32p = C.POINTER(C.c_int32)
c_i16p = C.POINTER(C.c_int16)
c_i8p = C.POINTER(C.c_int8)
c_u16p = C.POINTER(C.c_uint16)

ARM_MATH_SUCCESS = 0
ARM_MATH_ARGUMENT_ERROR = -1
ARM_MATH_LENGTH_ERROR = -2
ARM_MATH_SIZE_MISMATCH = -3


def _cfft_struct(name, twp):
    # Include/dsp/transform_functions.h:410-424 (scalar layout)
    return type(name, (C.Structure,), {"_fields_": [
        ("fftLen", C.c_uint16), ("pTwiddle", twp), ("pBitRevTable", c_u16p), ("bitRevLength", C.c_uint16)]})


arm_cfft_instance_f32 = _cfft_struct("arm_cfft_instance_f32", c_f32p)
arm_cfft_instance_q31 = _cfft_struct("arm_cfft_instance_q31", c_i32p)
arm_cfft_instance_q15 = _cfft_struct("arm_cfft_instance_q15", c_i16p)


class arm_rfft_fast_instance_f32(C.Structure):
    # Include/dsp/transform_functions.h:813-818
    _fields_ = [("Sint", arm_cfft_instance_f32), ("fftLenRFFT", C.c_uint16), ("pTwiddleRFFT", c_f32p)]


def _rfft_fixed_struct(name, twp, cfft):
    # Include/dsp/transform_functions.h:636-649 (q31), :508-521 (q15): non-Neon, non-MVE layout
    return type(name, (C.Structure,), {"_fields_": [
        ("fftLenReal", C.c_uint32), ("ifftFlagR", C.c_uint8), ("bitReverseFlagR", C.c_uint8),
        ("twidCoefRModifier", C.c_uint32), ("pTwiddleAReal", twp), ("pTwiddleBReal", twp),
        ("pCfft", C.POINTER(cfft))]})


arm_rfft_instance_q31 = _rfft_fixed_struct("arm_rfft_instance_q31", c_i32p, arm_cfft_instance_q31)
arm_rfft_instance_q15 = _rfft_fixed_struct("arm_rfft_instance_q15", c_i16p, arm_cfft_instance_q15)


class arm_fir_instance_f32(C.Structure):
    # Include/dsp/filtering_functions.h:86-91
    _fields_ = [("numTaps", C.c_uint16), ("pState", c_f32p), ("pCoeffs", c_f32p)]


class arm_fir_instance_q7(C.Structure):
    _fields_ = [("numTaps", C.c_uint16), ("pState", C.c_void_p), ("pCoeffs", C.c_void_p)]


# arm_fir_decimate_instance_{f32,q15,q31} / arm_fir_interpolate_instance_{f32,q15,q31}: one
# layout per family (the element type only changes the pointees)
class arm_fir_decimate_instance(C.Structure):
    _fields_ = [("M", C.c_uint8), ("numTaps", C.c_uint16), ("pCoeffs", C.c_void_p), ("pState", C.c_void_p)]


class arm_fir_interpolate_instance(C.Structure):
    _fields_ = [("L", C.c_uint8), ("phaseLength", C.c_uint16), ("pCoeffs", C.c_void_p), ("pState", C.c_void_p)]


# arm_fir_lattice_instance_{f32,q31,q15} (filtering_functions.h:1312-1340), one layout
class arm_fir_lattice_instance(C.Structure):
    _fields_ = [("numStages", C.c_uint16), ("pState", C.c_void_p), ("pCoeffs", C.c_void_p)]


# arm_fir_sparse_instance_{f32,q31,q15,q7} (filtering_functions.h:2033-2091), one layout
class arm_fir_sparse_instance(C.Structure):
    _fields_ = [("numTaps", C.c_uint16), ("stateIndex", C.c_uint16), ("pState", C.c_void_p), ("pCoeffs", C.c_void_p),
                ("maxDelay", C.c_uint16), ("pTapDelay", C.c_void_p)]


class arm_fir_instance_q15(C.Structure):
    # Include/dsp/filtering_functions.h:66-71
    _fields_ = [("numTaps", C.c_uint16), ("pState", c_i16p), ("pCoeffs", c_i16p)]


class arm_fir_instance_q31(C.Structure):
    # Include/dsp/filtering_functions.h:76-81
    _fields_ = [("numTaps", C.c_uint16), ("pState", c_i32p), ("pCoeffs", c_i32p)]


class arm_matrix_instance_f32(C.Structure):
    # Include/dsp/matrix_functions.h:118-123
    _fields_ = [("numRows", C.c_uint16), ("numCols", C.c_uint16), ("pData", c_f32p)]


class arm_mfcc_instance_f32(C.Structure):
    # Include/dsp/transform_functions.h:856-873 (RFFT-based default build)
    _fields_ = [("dctCoefs", c_f32p), ("filterCoefs", c_f32p), ("windowCoefs", c_f32p),
                ("filterPos", C.POINTER(C.c_uint32)), ("filterLengths", C.POINTER(C.c_uint32)),
                ("fftLen", C.c_uint32), ("nbMelFilters", C.c_uint32), ("nbDctOutputs", C.c_uint32),
                ("rfft", arm_rfft_fast_instance_f32)]


class arm_mfcc_instance_q31(C.Structure):
    # Include/dsp/transform_functions.h:1000-1020 (RFFT-based default build)
    _fields_ = [("dctCoefs", c_i32p), ("filterCoefs", c_i32p), ("windowCoefs", c_i32p),
                ("filterPos", C.POINTER(C.c_uint32)), ("filterLengths", C.POINTER(C.c_uint32)),
                ("fftLen", C.c_uint32), ("nbMelFilters", C.c_uint32), ("nbDctOutputs", C.c_uint32),
                ("rfft", arm_rfft_instance_q31)]


class arm_mfcc_instance_q15(C.Structure):
    # Include/dsp/transform_functions.h:1150-1168 (RFFT-based default build)
    _fields_ = [("dctCoefs", c_i16p), ("filterCoefs", c_i16p), ("windowCoefs", c_i16p),
                ("filterPos", C.POINTER(C.c_uint32)), ("filterLengths", C.POINTER(C.c_uint32)),
                ("fftLen", C.c_uint32), ("nbMelFilters", C.c_uint32), ("nbDctOutputs", C.c_uint32),
                ("rfft", arm_rfft_instance_q15)]


class arm_matrix_instance_q7(C.Structure):
    # Include/dsp/matrix_functions.h:139-143
    _fields_ = [("numRows", C.c_uint16), ("numCols", C.c_uint16), ("pData", c_i8p)]


class arm_matrix_instance_q15(C.Structure):
    # Include/dsp/matrix_functions.h:139-144
    _fields_ = [("numRows", C.c_uint16), ("numCols", C.c_uint16), ("pData", c_i16p)]


class arm_matrix_instance_q31(C.Structure):
    # Include/dsp/matrix_functions.h:149-154
    _fields_ = [("numRows", C.c_uint16), ("numCols", C.c_uint16), ("pData", c_i32p)]


P = C.POINTER
SIZES = (16, 32, 64, 128, 256, 512, 1024, 2048, 4096)
RFFT_SIZES = (32, 64, 128, 256, 512, 1024, 2048, 4096)
# convolution / correlation family (drop-in names without the arm_ prefix)
CONV_FULL = ("conv_f32", "conv_q15", "conv_q31", "conv_fast_q15", "conv_fast_q31", "correlate_f32", "correlate_q15",
             "correlate_q31", "correlate_fast_q15", "correlate_fast_q31", "conv_q7", "correlate_q7")
CONV_PARTIAL = ("conv_partial_f32", "conv_partial_q15", "conv_partial_q31", "conv_partial_q7")
# product only (the oracle restates them as arm_conv_fast_* over the range; the reference's
# own bodies are memory-unsafe for most ranges)
CONV_PARTIAL_FAST = ("conv_partial_fast_q15", "conv_partial_fast_q31")
# scratch-buffer forms: name -> number of trailing scratch pointers
CONV_OPT_FULL = {"conv_opt_q15": 2, "conv_fast_opt_q15": 2, "conv_opt_q7": 2, "correlate_opt_q15": 1,
                 "correlate_fast_opt_q15": 1, "correlate_opt_q7": 2}
CONV_OPT_PARTIAL = ("conv_partial_opt_q15", "conv_partial_fast_opt_q15", "conv_partial_opt_q7")

# name -> (restype, argtypes): the drop-in surface of include/arm_math.h
DROPIN = {
    "arm_cfft_init_f32": (C.c_int, [P(arm_cfft_instance_f32), C.c_uint16]),
    "arm_cfft_init_q31": (C.c_int, [P(arm_cfft_instance_q31), C.c_uint16]),
    "arm_cfft_init_q15": (C.c_int, [P(arm_cfft_instance_q15), C.c_uint16]),
    "arm_cfft_f32": (None, [P(arm_cfft_instance_f32), C.c_void_p, C.c_uint8, C.c_uint8]),
    "arm_cfft_q31": (None, [P(arm_cfft_instance_q31), C.c_void_p, C.c_uint8, C.c_uint8]),
    "arm_cfft_q15": (None, [P(arm_cfft_instance_q15), C.c_void_p, C.c_uint8, C.c_uint8]),
    "arm_rfft_fast_init_f32": (C.c_int, [P(arm_rfft_fast_instance_f32), C.c_uint16]),
    "arm_rfft_fast_f32": (None, [P(arm_rfft_fast_instance_f32), C.c_void_p, C.c_void_p, C.c_uint8]),
    "arm_rfft_init_q31": (C.c_int, [P(arm_rfft_instance_q31), C.c_uint32, C.c_uint32, C.c_uint32]),
    "arm_rfft_init_q15": (C.c_int, [P(arm_rfft_instance_q15), C.c_uint32, C.c_uint32, C.c_uint32]),
    "arm_rfft_q31": (None, [P(arm_rfft_instance_q31), C.c_void_p, C.c_void_p]),
    "arm_rfft_q15": (None, [P(arm_rfft_instance_q15), C.c_void_p, C.c_void_p]),
    "arm_fir_init_f32": (None, [P(arm_fir_instance_f32), C.c_uint16, C.c_void_p, C.c_void_p, C.c_uint32]),
    "arm_fir_f32": (None, [P(arm_fir_instance_f32), C.c_void_p, C.c_void_p, C.c_uint32]),
    "arm_fir_init_q15": (C.c_int, [P(arm_fir_instance_q15), C.c_uint16, C.c_void_p, C.c_void_p, C.c_uint32]),
    "arm_fir_q15": (None, [P(arm_fir_instance_q15), C.c_void_p, C.c_void_p, C.c_uint32]),
    "arm_fir_fast_q15": (None, [P(arm_fir_instance_q15), C.c_void_p, C.c_void_p, C.c_uint32]),
    "arm_fir_init_q31": (None, [P(arm_fir_instance_q31), C.c_uint16, C.c_void_p, C.c_void_p, C.c_uint32]),
    "arm_fir_q31": (None, [P(arm_fir_instance_q31), C.c_void_p, C.c_void_p, C.c_uint32]),
    "arm_fir_fast_q31": (None, [P(arm_fir_instance_q31), C.c_void_p, C.c_void_p, C.c_uint32]),
    "arm_fir_init_q7": (None, [P(arm_fir_instance_q7), C.c_uint16, C.c_void_p, C.c_void_p, C.c_uint32]),
    **{f"arm_fir_decimate_init_{t}": (C.c_int, [P(arm_fir_decimate_instance), C.c_uint16, C.c_uint8, C.c_void_p,
                                                C.c_void_p, C.c_uint32]) for t in ("f32", "q15", "q31")},
    **{f"arm_fir_interpolate_init_{t}": (C.c_int, [P(arm_fir_interpolate_instance), C.c_uint8, C.c_uint16,
                                                   C.c_void_p, C.c_void_p, C.c_uint32]) for t in ("f32", "q15", "q31")},
    **{f"arm_fir_{k}": (None, [P(arm_fir_decimate_instance), C.c_void_p, C.c_void_p, C.c_uint32])
       for k in ("decimate_f32", "decimate_q15", "decimate_fast_q15", "decimate_q31", "decimate_fast_q31")},
    **{f"arm_fir_{k}": (None, [P(arm_fir_interpolate_instance), C.c_void_p, C.c_void_p, C.c_uint32])
       for k in ("interpolate_f32", "interpolate_q15", "interpolate_q31")},
    "arm_fir_q7": (None, [P(arm_fir_instance_q7), C.c_void_p, C.c_void_p, C.c_uint32]),
    **{f"arm_{k}": (None, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p] + [C.c_void_p] * n)
       for k, n in CONV_OPT_FULL.items()},
    **{f"arm_{k}": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_uint32,
                              C.c_void_p, C.c_void_p]) for k in CONV_OPT_PARTIAL},
    **{f"arm_fir_lattice_init_{t}": (None, [P(arm_fir_lattice_instance), C.c_uint16, C.c_void_p, C.c_void_p])
       for t in ("f32", "q31", "q15")},
    **{f"arm_fir_lattice_{t}": (None, [P(arm_fir_lattice_instance), C.c_void_p, C.c_void_p, C.c_uint32])
       for t in ("f32", "q31", "q15")},
    **{f"arm_fir_sparse_init_{t}": (None, [P(arm_fir_sparse_instance), C.c_uint16, C.c_void_p, C.c_void_p, C.c_void_p,
                                           C.c_uint16, C.c_uint32]) for t in ("f32", "q31", "q15", "q7")},
    **{f"arm_fir_sparse_{t}": (None, [P(arm_fir_sparse_instance), C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32])
       for t in ("f32", "q31")},
    **{f"arm_fir_sparse_{t}": (None, [P(arm_fir_sparse_instance), C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                      C.c_uint32]) for t in ("q15", "q7")},
    "arm_mat_init_f32": (None, [P(arm_matrix_instance_f32), C.c_uint16, C.c_uint16, C.c_void_p]),
    "arm_mat_init_q7": (None, [P(arm_matrix_instance_q7), C.c_uint16, C.c_uint16, C.c_void_p]),
    "arm_mat_init_q15": (None, [P(arm_matrix_instance_q15), C.c_uint16, C.c_uint16, C.c_void_p]),
    "arm_mat_mult_q7": (C.c_int, [P(arm_matrix_instance_q7), P(arm_matrix_instance_q7),
                                  P(arm_matrix_instance_q7), C.c_void_p]),
    "arm_mat_init_q31": (None, [P(arm_matrix_instance_q31), C.c_uint16, C.c_uint16, C.c_void_p]),
    "arm_mat_mult_q15": (C.c_int, [P(arm_matrix_instance_q15), P(arm_matrix_instance_q15),
                                   P(arm_matrix_instance_q15), C.c_void_p]),
    "arm_mat_mult_q31": (C.c_int, [P(arm_matrix_instance_q31), P(arm_matrix_instance_q31),
                                   P(arm_matrix_instance_q31)]),
    "arm_mat_mult_opt_q31": (C.c_int, [P(arm_matrix_instance_q31), P(arm_matrix_instance_q31),
                                       P(arm_matrix_instance_q31), C.c_void_p]),
    "arm_mat_mult_fast_q15": (C.c_int, [P(arm_matrix_instance_q15), P(arm_matrix_instance_q15),
                                        P(arm_matrix_instance_q15), C.c_void_p]),
    "arm_mat_mult_fast_q31": (C.c_int, [P(arm_matrix_instance_q31), P(arm_matrix_instance_q31),
                                        P(arm_matrix_instance_q31)]),
    "arm_conv_f32": (None, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p]),
    "arm_conv_q15": (None, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p]),
    "arm_conv_q31": (None, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p]),
    **{f"arm_{f}": (None, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p])
       for f in CONV_FULL if f not in ("conv_f32", "conv_q15", "conv_q31")},
    **{f"arm_{f}": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_uint32])
       for f in CONV_PARTIAL},
    "arm_mfcc_init_f32": (C.c_int, [P(arm_mfcc_instance_f32), C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p,
                                    C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "arm_mfcc_f32": (None, [P(arm_mfcc_instance_f32), C.c_void_p, C.c_void_p, C.c_void_p]),
    "arm_mfcc_init_q31": (C.c_int, [P(arm_mfcc_instance_q31), C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p,
                                    C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "arm_mfcc_q31": (C.c_int, [P(arm_mfcc_instance_q31), C.c_void_p, C.c_void_p, C.c_void_p]),
    "arm_mfcc_init_q15": (C.c_int, [P(arm_mfcc_instance_q15), C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p,
                                    C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "arm_mfcc_q15": (C.c_int, [P(arm_mfcc_instance_q15), C.c_void_p, C.c_void_p, C.c_void_p]),
    "arm_mat_mult_f32": (C.c_int, [P(arm_matrix_instance_f32), P(arm_matrix_instance_f32),
                                   P(arm_matrix_instance_f32)]),
}
for _t in ("f32", "q31", "q15"):
    _inst = {"f32": arm_cfft_instance_f32, "q31": arm_cfft_instance_q31, "q15": arm_cfft_instance_q15}[_t]
    for _n in SIZES:
        DROPIN[f"arm_cfft_init_{_n}_{_t}"] = (C.c_int, [P(_inst)])
for _n in RFFT_SIZES:
    DROPIN[f"arm_rfft_fast_init_{_n}_f32"] = (C.c_int, [P(arm_rfft_fast_instance_f32)])

# per-length MFCC init functions (the product and the reference build; the oracle has the
# generic init only)
MFCC_LEN = {f"arm_mfcc_init_{n}_f32": (C.c_int, [P(arm_mfcc_instance_f32), C.c_uint32, C.c_uint32, C.c_void_p,
                                                 C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p])
            for n in RFFT_SIZES}
MFCC_LEN.update({f"arm_mfcc_init_{n}_q31": (C.c_int, [P(arm_mfcc_instance_q31), C.c_uint32, C.c_uint32, C.c_void_p,
                                                      C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p])
                 for n in RFFT_SIZES})
MFCC_LEN.update({f"arm_mfcc_init_{n}_q15": (C.c_int, [P(arm_mfcc_instance_q15), C.c_uint32, C.c_uint32, C.c_void_p,
                                                      C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p])
                 for n in RFFT_SIZES})

# per-length q31 / q15 RFFT init functions (product and reference build; the oracle has
# the generic init only)
RFFTQ_SIZES = (32, 64, 128, 256, 512, 1024, 2048, 4096, 8192)
RFFTQ_LEN = {f"arm_rfft_init_{n}_{t}": (C.c_int, [P(arm_rfft_instance_q31 if t == "q31" else arm_rfft_instance_q15),
                                                 C.c_uint32, C.c_uint32])
             for n in RFFTQ_SIZES for t in ("q31", "q15")}

PARTIAL_FAST = {f"arm_{f}": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32,
                                       C.c_uint32]) for f in CONV_PARTIAL_FAST}

# the additive batched device API of include/arm_math_mi355x.h
BATCHED = {
    "arm_cfft_f32_batch": (C.c_int, [P(arm_cfft_instance_f32), C.c_void_p, C.c_uint32, C.c_uint8, C.c_uint8,
                                     C.c_void_p]),
    "arm_cfft_q31_batch": (C.c_int, [P(arm_cfft_instance_q31), C.c_void_p, C.c_uint32, C.c_uint8, C.c_uint8,
                                     C.c_void_p]),
    "arm_cfft_q15_batch": (C.c_int, [P(arm_cfft_instance_q15), C.c_void_p, C.c_uint32, C.c_uint8, C.c_uint8,
                                     C.c_void_p]),
    "arm_rfft_fast_f32_batch": (C.c_int, [P(arm_rfft_fast_instance_f32), C.c_void_p, C.c_void_p, C.c_uint32,
                                          C.c_uint8, C.c_void_p]),
    "arm_rfft_fast_f32_batch_ex": (C.c_int, [P(arm_rfft_fast_instance_f32), C.c_void_p, C.c_void_p, C.c_uint32,
                                             C.c_uint8, C.c_uint32, C.c_void_p]),
    "arm_rfft_q31_batch": (C.c_int, [P(arm_rfft_instance_q31), C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p]),
    "arm_rfft_q15_batch": (C.c_int, [P(arm_rfft_instance_q15), C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p]),
    "arm_fir_f32_batch": (C.c_int, [P(arm_fir_instance_f32), C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32,
                                    C.c_void_p, C.c_void_p]),
    "arm_fir_f32_batch_fma": (C.c_int, [P(arm_fir_instance_f32), C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32,
                                        C.c_void_p, C.c_void_p]),
    "arm_fir_q15_batch": (C.c_int, [P(arm_fir_instance_q15), C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32,
                                    C.c_void_p, C.c_void_p]),
    "arm_fir_fast_q15_batch": (C.c_int, [P(arm_fir_instance_q15), C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32,
                                         C.c_void_p, C.c_void_p]),
    "arm_fir_q31_batch": (C.c_int, [P(arm_fir_instance_q31), C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32,
                                    C.c_void_p, C.c_void_p]),
    "arm_fir_fast_q31_batch": (C.c_int, [P(arm_fir_instance_q31), C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32,
                                         C.c_void_p, C.c_void_p]),
    "arm_fir_q7_batch": (C.c_int, [P(arm_fir_instance_q7), C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32,
                                   C.c_void_p, C.c_void_p]),
    **{f"arm_fir_{k}_batch": (C.c_int, [P(arm_fir_decimate_instance), C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32,
                                        C.c_void_p, C.c_void_p])
       for k in ("decimate_f32", "decimate_q15", "decimate_fast_q15", "decimate_q31", "decimate_fast_q31")},
    **{f"arm_fir_{k}_batch": (C.c_int, [P(arm_fir_interpolate_instance), C.c_void_p, C.c_void_p, C.c_uint32,
                                        C.c_uint32, C.c_void_p, C.c_void_p])
       for k in ("interpolate_f32", "interpolate_q15", "interpolate_q31")},
    **{f"arm_fir_lattice_{t}_batch": (C.c_int, [P(arm_fir_lattice_instance), C.c_void_p, C.c_void_p, C.c_uint32,
                                                C.c_uint32, C.c_void_p, C.c_void_p]) for t in ("f32", "q31", "q15")},
    **{f"arm_fir_sparse_{t}_batch": (C.c_int, [P(arm_fir_sparse_instance), C.c_void_p, C.c_void_p, C.c_uint32,
                                               C.c_uint32, C.c_void_p, C.c_void_p]) for t in ("f32", "q31", "q15", "q7")},
    "arm_mat_mult_f32_batch": (C.c_int, [P(arm_matrix_instance_f32), P(arm_matrix_instance_f32),
                                         P(arm_matrix_instance_f32), C.c_uint32, C.c_void_p]),
    "arm_mat_mult_q7_batch": (C.c_int, [P(arm_matrix_instance_q7), P(arm_matrix_instance_q7),
                                        P(arm_matrix_instance_q7), C.c_uint32, C.c_void_p]),
    "arm_mat_mult_q15_batch": (C.c_int, [P(arm_matrix_instance_q15), P(arm_matrix_instance_q15),
                                         P(arm_matrix_instance_q15), C.c_uint32, C.c_void_p]),
    "arm_mat_mult_q31_batch": (C.c_int, [P(arm_matrix_instance_q31), P(arm_matrix_instance_q31),
                                         P(arm_matrix_instance_q31), C.c_uint32, C.c_void_p]),
    "arm_mat_mult_fast_q15_batch": (C.c_int, [P(arm_matrix_instance_q15), P(arm_matrix_instance_q15),
                                              P(arm_matrix_instance_q15), C.c_uint32, C.c_void_p]),
    "arm_mat_mult_fast_q31_batch": (C.c_int, [P(arm_matrix_instance_q31), P(arm_matrix_instance_q31),
                                              P(arm_matrix_instance_q31), C.c_uint32, C.c_void_p]),
    **{f"arm_{f}_batch": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint32, C.c_uint32,
                                    C.c_void_p, C.c_uint32, C.c_void_p]) for f in CONV_FULL},
    **{f"arm_{f}_batch": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint32, C.c_uint32,
                                    C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p])
       for f in CONV_PARTIAL + CONV_PARTIAL_FAST},
    "arm_mfcc_f32_batch": (C.c_int, [P(arm_mfcc_instance_f32), C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                     C.c_void_p]),
    "arm_mfcc_q31_batch": (C.c_int, [P(arm_mfcc_instance_q31), C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                     C.c_void_p]),
    "arm_mfcc_q15_batch": (C.c_int, [P(arm_mfcc_instance_q15), C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                     C.c_void_p]),
    **{f"arm_cfft_{t}_batch_multi": (C.c_int, [P(inst), C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p,
                                               C.c_uint8, C.c_uint8])
       for t, inst in (("f32", arm_cfft_instance_f32), ("q31", arm_cfft_instance_q31),
                       ("q15", arm_cfft_instance_q15))},
    **{f"arm_fir_{t}_batch_multi": (C.c_int, [P(inst), C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                              C.c_uint32, C.c_void_p])
       for t, inst in (("f32", arm_fir_instance_f32), ("q15", arm_fir_instance_q15), ("fast_q15", arm_fir_instance_q15),
                       ("q31", arm_fir_instance_q31), ("fast_q31", arm_fir_instance_q31), ("q7", arm_fir_instance_q7))},
    **{f"arm_mat_mult_{t}_batch_multi": (C.c_int, [P(inst), P(inst), P(inst), C.c_uint32, C.c_void_p, C.c_void_p,
                                                   C.c_void_p, C.c_void_p, C.c_void_p])
       for t, inst in (("f32", arm_matrix_instance_f32), ("q15", arm_matrix_instance_q15),
                       ("q31", arm_matrix_instance_q31), ("q7", arm_matrix_instance_q7))},
    "arm_mi355x_device_count": (C.c_int, []),
    "arm_mi355x_last_error": (C.c_int, []),
    "arm_mi355x_last_error_string": (C.c_char_p, []),
    "arm_mi355x_clear_error": (None, []),
    "arm_mi355x_version": (C.c_char_p, []),
    "arm_mi355x_table_cache_bytes": (C.c_size_t, []),
    "arm_mi355x_set_table_cache_limit": (None, [C.c_size_t]),
    "arm_mi355x_release_thread_resources": (None, []),
    "arm_mi355x_thread_resource_owners": (C.c_int, []),
}

# exported data symbols (arm_const_structs.h / arm_common_tables.h)
DATA = ([f"arm_cfft_sR_{t}_len{n}" for t in ("f32", "q31", "q15") for n in SIZES]
        + [f"arm_rfft_fast_sR_f32_len{n}" for n in RFFT_SIZES]
        + [f"twiddleCoef_{n}" for n in SIZES] + [f"twiddleCoef_{n}_q31" for n in SIZES]
        + [f"twiddleCoef_{n}_q15" for n in SIZES] + [f"twiddleCoef_rfft_{n}" for n in RFFT_SIZES]
        + [f"armBitRevIndexTable{n}" for n in SIZES] + [f"armBitRevIndexTable_fixed_{n}" for n in SIZES])


def bind(lib, table, prefix=""):
    """Attach restype/argtypes for every function of `table` (optionally name-prefixed)."""
    for name, (res, args) in table.items():
        fn = getattr(lib, prefix + name)
        fn.restype = res
        fn.argtypes = args
    return lib
