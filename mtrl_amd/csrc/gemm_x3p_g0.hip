// gemm_x3p_g0.hip -- instantiation unit of the plane GEMM: GeoSmall, operand-form mask 15
#include "gemm_x3p_impl.h"

namespace mtsac {
X3P_UNIT(x3p_unit_g0, GeoSmall, 15)
}  // namespace mtsac
