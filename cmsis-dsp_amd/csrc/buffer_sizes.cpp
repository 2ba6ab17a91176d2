// Transform buffer-size helpers of the reference C API (host only, no device work).
// Reference: Include/dsp/transform_functions.h:1307-1398 (prototypes), Include/arm_math_types.h:
// 667-700 (arm_math_datatype / arm_math_target_arch), bodies in
// Source/TransformFunctions/arm_transform_buffer_sizes.c:47-330.  They answer "how many real
// elements does buffer X of transform Y need on target Z"; a C application that sizes its buffers
// with them links against this library unchanged.  Values are reproduced for every target the
// reference describes (the scalar build asks with ARM_MATH_SCALAR_ARCH, the default target).
// Lengths are computed in uint32_t as the reference does (2 * n wraps for n >= 2^31).
#include "../../include/arm_math.h"

namespace {

bool is_float(arm_math_datatype dt) { return dt == ARM_MATH_F16 || dt == ARM_MATH_F32 || dt == ARM_MATH_F64; }
bool is_fixed(arm_math_datatype dt) { return dt == ARM_MATH_Q31 || dt == ARM_MATH_Q15; }
int32_t words(uint32_t n) { return (int32_t)n; }

}  // namespace

extern "C" {

// Only the Neon CFFTs take a scratch buffer (buffer 1, one complex per sample); f64 and q7 have
// no Neon CFFT.
int32_t arm_cfft_tmp_buffer_size(arm_math_target_arch arch, arm_math_datatype dt, uint32_t nb_samples,
                                 uint32_t buf_id) {
  const bool neon_scratch = arch == ARM_MATH_NEON_ARCH && buf_id == 1 &&
                            (dt == ARM_MATH_F16 || dt == ARM_MATH_F32 || is_fixed(dt));
  return neon_scratch ? words(2u * nb_samples) : 0;
}

// A complex transform's output is nb_samples complex values on every target and type.
int32_t arm_cfft_output_buffer_size(arm_math_target_arch, arm_math_datatype, uint32_t nb_samples) {
  return words(2u * nb_samples);
}
int32_t arm_cifft_output_buffer_size(arm_math_target_arch, arm_math_datatype, uint32_t nb_samples) {
  return words(2u * nb_samples);
}

// RFFT / RIFFT scratch: Neon only, buffer 1: nb_samples reals for f16/f32, 2 nb_samples for
// q31/q15.  f64 and q7 need none.
int32_t arm_rfft_tmp_buffer_size(arm_math_target_arch arch, arm_math_datatype dt, uint32_t nb_samples,
                                 uint32_t buf_id) {
  if (arch != ARM_MATH_NEON_ARCH || buf_id != 1) return 0;
  if (dt == ARM_MATH_F16 || dt == ARM_MATH_F32) return words(nb_samples);
  if (is_fixed(dt)) return words(2u * nb_samples);
  return 0;
}

// RFFT output: nb_samples packed reals for the float types; the fixed-point RFFTs write the
// whole 2 nb_samples spectrum on the scalar and DSP targets and nb_samples + 2 on Helium / Neon.
int32_t arm_rfft_output_buffer_size(arm_math_target_arch arch, arm_math_datatype dt, uint32_t nb_samples) {
  if (is_float(dt)) return words(nb_samples);
  if (is_fixed(dt))
    return (arch == ARM_MATH_NEON_ARCH || arch == ARM_MATH_HELIUM_ARCH) ? words(nb_samples + 2u)
                                                                        : words(2u * nb_samples);
  return 0;
}

// RIFFT input: nb_samples packed reals (float) or nb_samples + 2 (q31/q15), on every target.
int32_t arm_rifft_input_buffer_size(arm_math_target_arch, arm_math_datatype dt, uint32_t nb_samples) {
  if (is_float(dt)) return words(nb_samples);
  if (is_fixed(dt)) return words(nb_samples + 2u);
  return 0;
}

// MFCC scratch: buffer 1 holds the transform output (CFFT-based or RFFT-based build), buffer 2
// (Neon only) the RFFT's own scratch.  The Neon MFCC is RFFT-based only: asking it for the CFFT
// form is the configuration error -1.
int32_t arm_mfcc_tmp_buffer_size(arm_math_target_arch arch, arm_math_datatype dt, uint32_t nb_samples,
                                 uint32_t buf_id, uint32_t use_cfft) {
  const bool neon = arch == ARM_MATH_NEON_ARCH;
  if (neon && use_cfft == 1) return -1;
  if (buf_id == 1)
    return use_cfft == 1 ? arm_cfft_output_buffer_size(arch, dt, nb_samples)
                         : arm_rfft_output_buffer_size(arch, dt, nb_samples);
  if (buf_id == 2 && neon) return arm_rfft_tmp_buffer_size(arch, dt, nb_samples, 1);
  return 0;
}

}  // extern "C"
