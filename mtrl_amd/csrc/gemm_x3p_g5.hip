// gemm_x3p_g5.hip -- instantiation unit of the plane GEMM: GeoTall224, row-major A forms (mask 5)
#include "gemm_x3p_impl.h"

namespace mtsac {
X3P_UNIT(x3p_unit_g5, GeoTall224, 5)
}  // namespace mtsac
