// v4 fused Informer instances for the P_X3 operand policy (cet_informer4.hpp; one precision per
// translation unit so the instances compile in parallel).
#include "cet_informer4.hpp"

extern "C" int cet_launch_informer_v4_p1(const cet::InformerArgs* a, int dff, int lds_bytes, hipStream_t stream) {
  return cet::v4::launch_v4<cet::v4::P_X3>(a, dff, lds_bytes, stream);
}

