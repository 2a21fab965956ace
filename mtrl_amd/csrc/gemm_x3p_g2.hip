// gemm_x3p_g2.hip -- instantiation unit of the plane GEMM: GeoWide16, operand-form mask 15
#include "gemm_x3p_impl.h"

namespace mtsac {
X3P_UNIT(x3p_unit_g2, GeoWide16, 15)
}  // namespace mtsac
