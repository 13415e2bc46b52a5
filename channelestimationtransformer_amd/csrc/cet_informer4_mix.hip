// v4 fused Informer instances of the mixed policy (host precision 4): the bf16 encoder with a split-bf16 decoder
// (cet_informer4.hpp PDEC; its own translation unit so the instances compile in parallel).
#include "cet_informer4.hpp"

extern "C" int cet_launch_informer_v4_p4(const cet::InformerArgs* a, int dff, int lds_bytes, hipStream_t stream) {
  return cet::v4::launch_v4_mix(a, dff, lds_bytes, stream);
}
