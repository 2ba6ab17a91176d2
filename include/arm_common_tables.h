/*
 * arm_common_tables.h — the CommonTables data the hot path consumes, exported by
 * libcmsisdsp_mi355x.so under the reference's symbol names
 * (Include/arm_common_tables.h:61-149, 181-236).  The words are the reference's own
 * (harvested, see cmsis-dsp_amd/tables/MANIFEST.json); they are embedded with .incbin
 * by cmsis-dsp_amd/csrc/tables_data.S.
 */
#ifndef ARM_COMMON_TABLES_MI355X_H
#define ARM_COMMON_TABLES_MI355X_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ARM_MI355X_DECL_FFT_TABLES(N)                                     \
  extern const float    twiddleCoef_##N[2 * (N)];                        \
  extern const int32_t  twiddleCoef_##N##_q31[3 * (N) / 2];              \
  extern const int16_t  twiddleCoef_##N##_q15[3 * (N) / 2];

ARM_MI355X_DECL_FFT_TABLES(16)
ARM_MI355X_DECL_FFT_TABLES(32)
ARM_MI355X_DECL_FFT_TABLES(64)
ARM_MI355X_DECL_FFT_TABLES(128)
ARM_MI355X_DECL_FFT_TABLES(256)
ARM_MI355X_DECL_FFT_TABLES(512)
ARM_MI355X_DECL_FFT_TABLES(1024)
ARM_MI355X_DECL_FFT_TABLES(2048)
ARM_MI355X_DECL_FFT_TABLES(4096)
#undef ARM_MI355X_DECL_FFT_TABLES

extern const float twiddleCoef_rfft_32[32];
extern const float twiddleCoef_rfft_64[64];
extern const float twiddleCoef_rfft_128[128];
extern const float twiddleCoef_rfft_256[256];
extern const float twiddleCoef_rfft_512[512];
extern const float twiddleCoef_rfft_1024[1024];
extern const float twiddleCoef_rfft_2048[2048];
extern const float twiddleCoef_rfft_4096[4096];

/* real FFT split twiddles, q31 / q15 (Include/arm_common_tables.h:241-245) */
extern const int32_t realCoefAQ31[8192];
extern const int32_t realCoefBQ31[8192];
extern const int16_t realCoefAQ15[8192];
extern const int16_t realCoefBQ15[8192];

/* initial 1/sqrt estimates of arm_sqrt_q31 (Include/arm_common_tables.h:297) */
extern const int32_t sqrt_initial_lut_q31[32];

/* bit-reversal table lengths: Include/arm_common_tables.h:181-235 */
#define ARMBITREVINDEXTABLE_16_TABLE_LENGTH   ((uint16_t)20)
#define ARMBITREVINDEXTABLE_32_TABLE_LENGTH   ((uint16_t)48)
#define ARMBITREVINDEXTABLE_64_TABLE_LENGTH   ((uint16_t)56)
#define ARMBITREVINDEXTABLE_128_TABLE_LENGTH  ((uint16_t)208)
#define ARMBITREVINDEXTABLE_256_TABLE_LENGTH  ((uint16_t)440)
#define ARMBITREVINDEXTABLE_512_TABLE_LENGTH  ((uint16_t)448)
#define ARMBITREVINDEXTABLE_1024_TABLE_LENGTH ((uint16_t)1800)
#define ARMBITREVINDEXTABLE_2048_TABLE_LENGTH ((uint16_t)3808)
#define ARMBITREVINDEXTABLE_4096_TABLE_LENGTH ((uint16_t)4032)

#define ARMBITREVINDEXTABLE_FIXED_16_TABLE_LENGTH   ((uint16_t)12)
#define ARMBITREVINDEXTABLE_FIXED_32_TABLE_LENGTH   ((uint16_t)24)
#define ARMBITREVINDEXTABLE_FIXED_64_TABLE_LENGTH   ((uint16_t)56)
#define ARMBITREVINDEXTABLE_FIXED_128_TABLE_LENGTH  ((uint16_t)112)
#define ARMBITREVINDEXTABLE_FIXED_256_TABLE_LENGTH  ((uint16_t)240)
#define ARMBITREVINDEXTABLE_FIXED_512_TABLE_LENGTH  ((uint16_t)480)
#define ARMBITREVINDEXTABLE_FIXED_1024_TABLE_LENGTH ((uint16_t)992)
#define ARMBITREVINDEXTABLE_FIXED_2048_TABLE_LENGTH ((uint16_t)1984)
#define ARMBITREVINDEXTABLE_FIXED_4096_TABLE_LENGTH ((uint16_t)4032)

extern const uint16_t armBitRevIndexTable16[ARMBITREVINDEXTABLE_16_TABLE_LENGTH];
extern const uint16_t armBitRevIndexTable32[ARMBITREVINDEXTABLE_32_TABLE_LENGTH];
extern const uint16_t armBitRevIndexTable64[ARMBITREVINDEXTABLE_64_TABLE_LENGTH];
extern const uint16_t armBitRevIndexTable128[ARMBITREVINDEXTABLE_128_TABLE_LENGTH];
extern const uint16_t armBitRevIndexTable256[ARMBITREVINDEXTABLE_256_TABLE_LENGTH];
extern const uint16_t armBitRevIndexTable512[ARMBITREVINDEXTABLE_512_TABLE_LENGTH];
extern const uint16_t armBitRevIndexTable1024[ARMBITREVINDEXTABLE_1024_TABLE_LENGTH];
extern const uint16_t armBitRevIndexTable2048[ARMBITREVINDEXTABLE_2048_TABLE_LENGTH];
extern const uint16_t armBitRevIndexTable4096[ARMBITREVINDEXTABLE_4096_TABLE_LENGTH];

extern const uint16_t armBitRevIndexTable_fixed_16[ARMBITREVINDEXTABLE_FIXED_16_TABLE_LENGTH];
extern const uint16_t armBitRevIndexTable_fixed_32[ARMBITREVINDEXTABLE_FIXED_32_TABLE_LENGTH];
extern const uint16_t armBitRevIndexTable_fixed_64[ARMBITREVINDEXTABLE_FIXED_64_TABLE_LENGTH];
extern const uint16_t armBitRevIndexTable_fixed_128[ARMBITREVINDEXTABLE_FIXED_128_TABLE_LENGTH];
extern const uint16_t armBitRevIndexTable_fixed_256[ARMBITREVINDEXTABLE_FIXED_256_TABLE_LENGTH];
extern const uint16_t armBitRevIndexTable_fixed_512[ARMBITREVINDEXTABLE_FIXED_512_TABLE_LENGTH];
extern const uint16_t armBitRevIndexTable_fixed_1024[ARMBITREVINDEXTABLE_FIXED_1024_TABLE_LENGTH];
extern const uint16_t armBitRevIndexTable_fixed_2048[ARMBITREVINDEXTABLE_FIXED_2048_TABLE_LENGTH];
extern const uint16_t armBitRevIndexTable_fixed_4096[ARMBITREVINDEXTABLE_FIXED_4096_TABLE_LENGTH];

#ifdef __cplusplus
}
#endif
#endif
