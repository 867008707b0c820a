#include <cmath>
#include <cstdio>
#include <random>
extern "C" void sum3(float*, const float*, const float*, const float*, const float*, int);
extern "C" void sum5(float*, const float*, const float*, const float*, const float*, const float*, const float*, int);
extern "C" void acc(float*, const float*, float, int);
int main() {
  const int n = 1 << 16;
  std::mt19937 g(1); std::normal_distribution<float> d;
  static float a[n], b[n], c[n], dd[n], e[n], o[n], o2[n];
  for (int i = 0; i < n; ++i) { a[i] = d(g); b[i] = d(g); c[i] = d(g); dd[i] = d(g); e[i] = d(g); }
  const float h[5] = {1.0 / 16.0, 4.0 / 16.0, 6.0 / 16.0, 4.0 / 16.0, 1.0 / 16.0};
  sum3(o, a, b, c, h, n);
  int m_plain = 0, m_fma_chain = 0, m_fma_first = 0;
  for (int i = 0; i < n; ++i) {
    float plain = a[i] * h[2] + b[i] * h[3] + c[i] * h[4];
    volatile float t = a[i] * h[2];
    float chain = std::fmaf(c[i], h[4], std::fmaf(b[i], h[3], t));      // fma(c,fma(b,a*h))
    volatile float t2 = b[i] * h[3];
    float first = std::fmaf(c[i], h[4], std::fmaf(a[i], h[2], t2));     // fma(a,h2, b*h3)
    m_plain += o[i] == plain; m_fma_chain += o[i] == chain; m_fma_first += o[i] == first;
  }
  printf("sum3: plain %d chain %d first %d of %d\n", m_plain, m_fma_chain, m_fma_first, n);
  sum5(o, a, b, c, dd, e, h, n);
  int c1 = 0, c2 = 0;
  for (int i = 0; i < n; ++i) {
    volatile float t = a[i] * h[2];
    float chain = std::fmaf(e[i], h[4], std::fmaf(dd[i], h[3], std::fmaf(c[i], h[0], std::fmaf(b[i], h[1], t))));
    volatile float t2 = b[i] * h[1];
    float first = std::fmaf(e[i], h[4], std::fmaf(dd[i], h[3], std::fmaf(c[i], h[0], std::fmaf(a[i], h[2], t2))));
    c1 += o[i] == chain; c2 += o[i] == first;
  }
  printf("sum5: chain %d first %d of %d\n", c1, c2, n);
  for (int i = 0; i < n; ++i) o[i] = e[i];
  acc(o, a, h[1], n);
  int a1 = 0;
  for (int i = 0; i < n; ++i) a1 += o[i] == std::fmaf(a[i], h[1], e[i]);
  printf("acc: fma %d of %d\n", a1, n);
}
