// Thread-local error message + status helpers for the C-ABI.
#pragma once
#include <string>

#include "../../include/cfm.h"

namespace cfm {
cfm_status set_error(cfm_status s, const std::string& msg);
int calc_length(int T);
}  // namespace cfm
