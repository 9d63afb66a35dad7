// Plan blob layout (int32), shared by the host planner and the device orchestration.
#pragma once
#include <stdint.h>

namespace cfm {

enum {
  PH_KIND = 0,      // 1 = masked batch, 2 = padded batch, 3 = streaming chunk (forward_chunk)
  PH_NWIN = 1,      // front-end windows (packed chunks / padded utterances)
  PH_NATT = 2,      // attention blocks
  PH_NCONV = 3,     // conv blocks
  PH_ROWS = 4,      // encoder rows (N*C or B*T')
  PH_C = 5,         // chunk size (masked) / effective chunk (padded; T' for full attention)
  PH_L = 6,
  PH_R = 7,
  PH_W = 8,         // front-end window rows (8C+7 or T)
  PH_TOUT = 9,      // encoder rows per window (C or T')
  PH_PROWS = 10,    // relative-position rows (L+2C+R-1 or 2T'-1)
  PH_PANCHOR = 11,  // distance of P row 0 (C+L-1 or T'-1)
  PH_KVROWS = 12,   // KV stream rows (L+N*C+R or B*T')
  PH_GLUROWS = 13,  // GLU stream rows (7+N*C+7 or B*T')
  PH_KVOFF = 14,    // stream row of encoder row 0 in the KV stream (L or 0)
  PH_GLUOFF = 15,   // same for the GLU stream (7 or 0)
  PH_HEADER = 16
};
constexpr int PLAN_REC = 8;

inline int64_t plan_ints(int nwin, int natt, int nconv, int rows) {
  return PH_HEADER + (int64_t)PLAN_REC * (nwin + natt + nconv) + ((int64_t)rows + 3) / 4;
}
inline int64_t plan_meta_off(const int32_t*) { return PH_HEADER; }
inline int64_t plan_att_off(const int32_t* h) { return PH_HEADER + (int64_t)PLAN_REC * h[PH_NWIN]; }
inline int64_t plan_conv_off(const int32_t* h) { return plan_att_off(h) + (int64_t)PLAN_REC * h[PH_NATT]; }
inline int64_t plan_mask_off(const int32_t* h) { return plan_conv_off(h) + (int64_t)PLAN_REC * h[PH_NCONV]; }

}  // namespace cfm
