// Probe of the gfx950 block-scaled MFMA operand layout (v_mfma_scale_f32_16x16x128_f8f6f4, e4m3 A/B):
// random small integers packed under a layout hypothesis, compared with the host product; then the
// per-lane E8M0 scale semantics.  Build: hipcc --offload-arch=gfx950 -O2 mfma_scale_probe.hip -o probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
__global__ void k(const v8i* a, const v8i* b, const int* sa, const int* sb, v4f* c) {
  int l = threadIdx.x;
  v4f acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[l], b[l], acc, 0, 0, 0, sa[l], 0, sb[l]);
  c[l] = acc;
}
static unsigned char e4m3(int v) {
  static const unsigned char pos[5] = {0x00, 0x38, 0x40, 0x44, 0x48};
  return v >= 0 ? pos[v] : (unsigned char)(pos[-v] | 0x80);
}
// hypothesis h: k index of byte j of lane l
static int kmap(int h, int l, int j) {
  const int g = l >> 4;
  if (h == 0) return 32 * g + j;
  if (h == 1) return j < 16 ? 16 * g + j : 64 + 16 * g + (j - 16);
  return 8 * g + (j & 7) + 32 * (j >> 3);   // h == 2
}

// Which outputs does one lane's scale byte reach?  A and B all ones (e4m3 1.0); every scale 2^0 except
// lane L of A (or B) at 2^1: an output C[row][col] that includes the pairs of that lane's block reads
// 128 + (pairs scaled).
static void scale_reach(v8i* da, v8i* db, int* dsa, int* dsb, v4f* dc) {
  unsigned char ones[64][32];
  memset(ones, 0x38, sizeof ones);
  hipMemcpy(da, ones, sizeof ones, hipMemcpyHostToDevice);
  hipMemcpy(db, ones, sizeof ones, hipMemcpyHostToDevice);
  const int lanes[6] = {0, 5, 16, 37, 48, 63};
  for (int side = 0; side < 2; ++side)
    for (int t = 0; t < 6; ++t) {
      int sa[64], sb[64];
      for (int l = 0; l < 64; ++l) sa[l] = sb[l] = 127;
      (side ? sb : sa)[lanes[t]] = 128;
      hipMemcpy(dsa, sa, sizeof sa, hipMemcpyHostToDevice);
      hipMemcpy(dsb, sb, sizeof sb, hipMemcpyHostToDevice);
      hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, da, db, dsa, dsb, dc);
      float hc[64][4];
      hipMemcpy(hc, dc, sizeof hc, hipMemcpyDeviceToHost);
      printf("%s scale of lane %2d raised:", side ? "B" : "A", lanes[t]);
      int shown = 0;
      for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 4; ++r)
          if (hc[l][r] != 128.f && shown < 20) {
            printf(" C[%d][%d]=%g", (l >> 4) * 4 + r, l & 15, hc[l][r]);
            ++shown;
          }
      printf("%s\n", shown >= 20 ? " ..." : "");
    }
}
int main() {
  int A[16][128], B[128][16];
  srand(7);
  for (int i = 0; i < 16; ++i) for (int k = 0; k < 128; ++k) A[i][k] = rand() % 9 - 4;
  for (int k = 0; k < 128; ++k) for (int n = 0; n < 16; ++n) B[k][n] = rand() % 9 - 4;
  v8i *da, *db; int *dsa, *dsb; v4f* dc;
  hipMalloc(&da, 64 * 32); hipMalloc(&db, 64 * 32); hipMalloc(&dsa, 256); hipMalloc(&dsb, 256); hipMalloc(&dc, 64 * 16);
  for (int h = 0; h < 3; ++h) {
    for (int sc = 0; sc < 2; ++sc) {
      unsigned char ha[64][32], hb[64][32];
      int sa[64], sb[64];
      for (int l = 0; l < 64; ++l) {
        for (int j = 0; j < 32; ++j) {
          ha[l][j] = e4m3(A[l & 15][kmap(h, l, j)]);
          hb[l][j] = e4m3(B[kmap(h, l, j)][l & 15]);
        }
        sa[l] = sc ? 127 + (l * 7 + 3) % 3 : 127;          // E8M0: 2^(e-127)
        sb[l] = sc ? 127 + (l * 5 + 1) % 3 : 127;
      }
      hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice);
      hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
      hipMemcpy(dsa, sa, sizeof sa, hipMemcpyHostToDevice);
      hipMemcpy(dsb, sb, sizeof sb, hipMemcpyHostToDevice);
      hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, da, db, dsa, dsb, dc);
      float hc[64][4];
      hipMemcpy(hc, dc, sizeof hc, hipMemcpyDeviceToHost);
      for (int rule = 0; rule < 2; ++rule) {
        int bad = 0;
        for (int l = 0; l < 64; ++l)
          for (int r = 0; r < 4; ++r) {
            const int row = (l >> 4) * 4 + r, col = l & 15;
            double ref = 0;
            for (int ll = 0; ll < 64; ll += 16)
              for (int j = 0; j < 32; ++j) {
                const int kk = kmap(h, ll, j);      // the k carried by byte j of lane group ll/16
                const int blk = rule ? kk / 32 : ll / 16;
                const double s = sc ? (double)(1 << (sa[row + 16 * blk] - 127)) * (1 << (sb[col + 16 * blk] - 127)) : 1.0;
                ref += s * A[row][kk] * B[kk][col];
              }
            if (hc[l][r] != (float)ref) ++bad;
          }
        printf("data layout %d, scale rule %d (%s), scales %s: %d of 256 outputs differ\n", h, rule,
               rule ? "block = k/32, lane row+16*block" : "block = the lane group holding k", sc ? "random" : "unit", bad);
      }
    }
  }
  scale_reach(da, db, dsa, dsb, dc);
  return 0;
}
