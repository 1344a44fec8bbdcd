// T=3 tree tails over a 4-plane pair-sum code + (x0, x1, c): 7 leaves, each used once.
#include <stdio.h>
#include <stdint.h>
#include <string.h>
typedef unsigned __int128 u128;
static u128 CARE, TGT;
static u128 gate(u128 a, u128 b, u128 c, int f) {
  u128 r = 0, ONE = ~(u128)0;
  for (int m = 0; m < 8; m++) if (f >> m & 1) r |= ((m & 4) ? a : ONE ^ a) & ((m & 2) ? b : ONE ^ b) & ((m & 1) ? c : ONE ^ c);
  return r;
}
static int func_of(const u128* s, int k) {
  u128 stack[16]; int n = 1; stack[0] = CARE;
  for (int i = 0; i < k; i++) {
    int nn = 0; u128 tmp[16];
    for (int j = 0; j < n; j++) {
      u128 a = stack[j] & s[i], b = stack[j] & ~s[i];
      if ((a & TGT) && (a & ~TGT)) tmp[nn++] = a;
      if ((b & TGT) && (b & ~TGT)) tmp[nn++] = b;
    }
    n = nn; memcpy(stack, tmp, n * sizeof(u128));
    if (!n) return 1;
  }
  return 0;
}
typedef int (*plane_fn)(int a0, int a1, int b0, int b1);
static int e1_0(int a0,int a1,int b0,int b1){return a0^b0;} static int e1_1(int a0,int a1,int b0,int b1){return a0&b0;}
static int e1_2(int a0,int a1,int b0,int b1){return a1^b1;} static int e1_3(int a0,int a1,int b0,int b1){return a1&b1;}
static int e2_2(int a0,int a1,int b0,int b1){return a1^b1^(a0&b0);} static int e2_3(int a0,int a1,int b0,int b1){return (a1&b1)|(a1&(a0&b0))|(b1&(a0&b0));}
static int e3_2(int a0,int a1,int b0,int b1){return a1|b1;} 
static int e4_1(int a0,int a1,int b0,int b1){return a0|b0;}
static int search(const char* name, plane_fn* pf) {
  u128 sig[7] = {0}; CARE = TGT = 0;
  for (int r = 0; r < 128; r++) {
    int a = r & 3, b = (r >> 2) & 3, x = (r >> 4) & 3, c = r >> 6;
    int a0 = a & 1, a1 = a >> 1, b0 = b & 1, b1 = b >> 1;
    for (int i = 0; i < 4; i++) if (pf[i](a0, a1, b0, b1)) sig[i] |= (u128)1 << r;
    if (x & 1) sig[4] |= (u128)1 << r;
    if (x >> 1) sig[5] |= (u128)1 << r;
    if (c) sig[6] |= (u128)1 << r;
    if (!c || a + b >= 1) CARE |= (u128)1 << r;
    int S = a + b + x;
    if (S == 3 || (S == 4 && c)) TGT |= (u128)1 << r;
  }
  int found = 0;
  // structure (ii): F(g1(3 leaves), g2(3 leaves), leaf)
  for (int l = 0; l < 7; l++) {
    int rest[6], nr = 0; for (int i = 0; i < 7; i++) if (i != l) rest[nr++] = i;
    for (int m = 0; m < 64; m++) { if (__builtin_popcount(m) != 3 || !(m & 1)) continue;  // g1 holds rest[0]
      int A[3], B[3], na = 0, nb = 0;
      for (int i = 0; i < 6; i++) if (m >> i & 1) A[na++] = rest[i]; else B[nb++] = rest[i];
      for (int f1 = 0; f1 < 256; f1++) { u128 g1 = gate(sig[A[0]], sig[A[1]], sig[A[2]], f1);
        for (int f2 = 0; f2 < 256; f2++) { u128 g2 = gate(sig[B[0]], sig[B[1]], sig[B[2]], f2);
          u128 s3[3] = {g1, g2, sig[l]};
          if (func_of(s3, 3)) { if (found++ < 3) printf("%s (ii) g1(%d%d%d,%02x) g2(%d%d%d,%02x) leaf %d\n", name, A[0],A[1],A[2],f1,B[0],B[1],B[2],f2,l); }
        } } } }
  // structure (i): g1(3 leaves), g2(g1, 2 leaves), F(g2, 2 leaves)
  for (int m1 = 0; m1 < 128; m1++) { if (__builtin_popcount(m1) != 3) continue;
    int A[3], na = 0, rest[4], nr = 0; for (int i = 0; i < 7; i++) if (m1 >> i & 1) A[na++] = i; else rest[nr++] = i;
    for (int m2 = 0; m2 < 16; m2++) { if (__builtin_popcount(m2) != 2) continue;
      int B[2], C[2], nb = 0, nc = 0; for (int i = 0; i < 4; i++) if (m2 >> i & 1) B[nb++] = rest[i]; else C[nc++] = rest[i];
      for (int f1 = 0; f1 < 256; f1++) { u128 g1 = gate(sig[A[0]], sig[A[1]], sig[A[2]], f1);
        for (int f2 = 0; f2 < 256; f2++) { u128 g2 = gate(g1, sig[B[0]], sig[B[1]], f2);
          u128 s3[3] = {g2, sig[C[0]], sig[C[1]]};
          if (func_of(s3, 3)) { if (found++ < 6) printf("%s (i) g1(%d%d%d,%02x) g2(g1,%d%d,%02x) F(g2,%d,%d)\n", name, A[0],A[1],A[2],f1,B[0],B[1],f2,C[0],C[1]); }
        } } } }
  printf("%s: %d trees\n", name, found);
  return found;
}
int main() {
  plane_fn E1[4] = {e1_0, e1_1, e1_2, e1_3};
  plane_fn E2[4] = {e1_0, e1_1, e2_2, e2_3};
  plane_fn E3[4] = {e1_0, e1_1, e1_2, e3_2};
  plane_fn E4[4] = {e1_0, e4_1, e1_2, e1_3};
  search("half-adders (a0^b0, a0&b0, a1^b1, a1&b1)", E1);
  search("binary+carry (p0, k, p1, p2)", E2);
  search("(a0^b0, a0&b0, a1^b1, a1|b1)", E3);
  search("(a0^b0, a0|b0, a1^b1, a1&b1)", E4);
}
