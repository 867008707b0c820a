// probe: how g++ -O3 -march=x86-64-v3 contracts 3/4/5-term tap sums
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
extern "C" void sum3(float* o, const float* a, const float* b, const float* c, const float* h, int n) {
  for (int i = 0; i < n; ++i) o[i] = a[i] * h[2] + b[i] * h[3] + c[i] * h[4];
}
extern "C" void sum5(float* o, const float* a, const float* b, const float* c, const float* d, const float* e, const float* h, int n) {
  for (int i = 0; i < n; ++i) o[i] = a[i] * h[2] + b[i] * h[1] + c[i] * h[0] + d[i] * h[3] + e[i] * h[4];
}
extern "C" void acc(float* o, const float* a, float v, int n) {
  for (int i = 0; i < n; ++i) o[i] += a[i] * v;
}
