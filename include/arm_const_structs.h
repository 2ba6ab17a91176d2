/*
 * arm_const_structs.h — pre-initialised CFFT / RFFT instances, exported by
 * libcmsisdsp_mi355x.so under the reference's names (Include/arm_const_structs.h:51-79;
 * definitions in the reference: Source/CommonTables/arm_const_structs.c:79-300).
 * Apps pass them straight to arm_cfft_*(): `arm_cfft_f32(&arm_cfft_sR_f32_len1024, p, 0, 1)`.
 */
#ifndef ARM_CONST_STRUCTS_MI355X_H
#define ARM_CONST_STRUCTS_MI355X_H

#include "arm_math.h"
#include "arm_common_tables.h"

#ifdef __cplusplus
extern "C" {
#endif

#define ARM_MI355X_DECL_CFFT(N)                                 \
  extern const arm_cfft_instance_f32 arm_cfft_sR_f32_len##N;   \
  extern const arm_cfft_instance_q31 arm_cfft_sR_q31_len##N;   \
  extern const arm_cfft_instance_q15 arm_cfft_sR_q15_len##N;
ARM_MI355X_DECL_CFFT(16)
ARM_MI355X_DECL_CFFT(32)
ARM_MI355X_DECL_CFFT(64)
ARM_MI355X_DECL_CFFT(128)
ARM_MI355X_DECL_CFFT(256)
ARM_MI355X_DECL_CFFT(512)
ARM_MI355X_DECL_CFFT(1024)
ARM_MI355X_DECL_CFFT(2048)
ARM_MI355X_DECL_CFFT(4096)
#undef ARM_MI355X_DECL_CFFT

extern const arm_rfft_fast_instance_f32 arm_rfft_fast_sR_f32_len32;
extern const arm_rfft_fast_instance_f32 arm_rfft_fast_sR_f32_len64;
extern const arm_rfft_fast_instance_f32 arm_rfft_fast_sR_f32_len128;
extern const arm_rfft_fast_instance_f32 arm_rfft_fast_sR_f32_len256;
extern const arm_rfft_fast_instance_f32 arm_rfft_fast_sR_f32_len512;
extern const arm_rfft_fast_instance_f32 arm_rfft_fast_sR_f32_len1024;
extern const arm_rfft_fast_instance_f32 arm_rfft_fast_sR_f32_len2048;
extern const arm_rfft_fast_instance_f32 arm_rfft_fast_sR_f32_len4096;

#ifdef __cplusplus
}
#endif
#endif
