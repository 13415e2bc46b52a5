// v4 fused Informer instances for the P_BF16 operand policy (cet_informer4.hpp; one precision per
// translation unit so the instances compile in parallel).
#include "cet_informer4.hpp"

extern "C" int cet_launch_informer_v4_p0(const cet::InformerArgs* a, int dff, int lds_bytes, hipStream_t stream) {
  return cet::v4::launch_v4<cet::v4::P_BF16>(a, dff, lds_bytes, stream);
}

extern "C" int cet_launch_informer_v4_p1(const cet::InformerArgs* a, int dff, int lds_bytes, hipStream_t stream);
extern "C" int cet_launch_informer_v4_p2(const cet::InformerArgs* a, int dff, int lds_bytes, hipStream_t stream);
extern "C" int cet_launch_informer_v4_p4(const cet::InformerArgs* a, int dff, int lds_bytes, hipStream_t stream);

extern "C" int cet_launch_informer_v4(const cet::InformerArgs* a, int prec, int dff, int lds_bytes, hipStream_t stream) {
  switch (prec) {
    case cet::v4::P_BF16: return cet_launch_informer_v4_p0(a, dff, lds_bytes, stream);
    case cet::v4::P_X3: return cet_launch_informer_v4_p1(a, dff, lds_bytes, stream);
    case cet::v4::P_FP8: return cet_launch_informer_v4_p2(a, dff, lds_bytes, stream);
    case 4: return cet_launch_informer_v4_p4(a, dff, lds_bytes, stream);   // bf16 encoder, split-bf16 decoder
    default: return -3;
  }
}
