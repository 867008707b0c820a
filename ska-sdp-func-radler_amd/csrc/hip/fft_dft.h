// Complex arithmetic and register-resident radix-R DFT butterflies shared by
// the LDS-resident FFT engines (lds_fft.hip: runtime plans; fft_fast.hip:
// compile-time plans). Forward transforms, e^{-2 pi i jk/R}.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace rdl {

// Aligned to its size so that a complex element moves as one 8- or 16-byte
// access (global and LDS), never as two scalar halves.
template <typename T>
struct alignas(2 * sizeof(T)) Cx {
  T x, y;
};

template <typename T>
__device__ __forceinline__ Cx<T> Add(Cx<T> a, Cx<T> b) {
  return {a.x + b.x, a.y + b.y};
}
template <typename T>
__device__ __forceinline__ Cx<T> Sub(Cx<T> a, Cx<T> b) {
  return {a.x - b.x, a.y - b.y};
}
template <typename T>
__device__ __forceinline__ Cx<T> Mul(Cx<T> a, Cx<T> b) {
  return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x};
}
template <typename T>
__device__ __forceinline__ Cx<T> MulMinusI(Cx<T> a) {  // a * (-i)
  return {a.y, -a.x};
}
template <typename T>
__device__ __forceinline__ Cx<T> Conj(Cx<T> a) {
  return {a.x, -a.y};
}
template <typename T>
__device__ __forceinline__ Cx<T> Scale(Cx<T> a, T s) {
  return {a.x * s, a.y * s};
}

// ---- radix-R DFT (forward, e^{-2 pi i jk/R}) on registers
template <typename T, int R>
struct Dft;

template <typename T>
struct Dft<T, 2> {
  __device__ __forceinline__ static void Run(Cx<T>* a) {
    const Cx<T> t = a[1];
    a[1] = Sub(a[0], t);
    a[0] = Add(a[0], t);
  }
};

template <typename T>
struct Dft<T, 4> {
  __device__ __forceinline__ static void Run(Cx<T>* a) {
    const Cx<T> t0 = Add(a[0], a[2]), t1 = Sub(a[0], a[2]);
    const Cx<T> t2 = Add(a[1], a[3]), t3 = MulMinusI(Sub(a[1], a[3]));
    a[0] = Add(t0, t2);
    a[2] = Sub(t0, t2);
    a[1] = Add(t1, t3);
    a[3] = Sub(t1, t3);
  }
};

template <typename T>
struct Dft<T, 8> {
  __device__ __forceinline__ static void Run(Cx<T>* a) {
    Cx<T> e[4] = {a[0], a[2], a[4], a[6]};
    Cx<T> o[4] = {a[1], a[3], a[5], a[7]};
    Dft<T, 4>::Run(e);
    Dft<T, 4>::Run(o);
    const T c = T(0.70710678118654752440084436210485);
    // o[k] *= W8^k, W8 = (c, -c)
    o[1] = {c * (o[1].x + o[1].y), c * (o[1].y - o[1].x)};
    o[2] = MulMinusI(o[2]);
    o[3] = {c * (o[3].y - o[3].x), -c * (o[3].x + o[3].y)};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      a[k] = Add(e[k], o[k]);
      a[k + 4] = Sub(e[k], o[k]);
    }
  }
};

// odd radix: pairs (a_j, a_{R-j})
template <int R>
struct OddTables;
template <>
struct OddTables<3> {
  static constexpr double c[3] = {1.0, -0.5, -0.5};
  static constexpr double s[3] = {0.0, 0.86602540378443864676372317075294,
                                  -0.86602540378443864676372317075294};
};
template <>
struct OddTables<5> {
  static constexpr double c[5] = {1.0, 0.30901699437494742410229341718282,
                                  -0.80901699437494742410229341718282,
                                  -0.80901699437494742410229341718282,
                                  0.30901699437494742410229341718282};
  static constexpr double s[5] = {0.0, 0.95105651629515357211643933337938,
                                  0.58778525229247312916870595463907,
                                  -0.58778525229247312916870595463907,
                                  -0.95105651629515357211643933337938};
};
template <>
struct OddTables<7> {
  static constexpr double c[7] = {1.0,
                                  0.62348980185873353052500488400424,
                                  -0.22252093395631440428890256449679,
                                  -0.90096886790241912623610231950745,
                                  -0.90096886790241912623610231950745,
                                  -0.22252093395631440428890256449679,
                                  0.62348980185873353052500488400424};
  static constexpr double s[7] = {0.0,
                                  0.78183148246802980870844452667406,
                                  0.97492791218182360701813168299393,
                                  0.43388373911755812047576833284836,
                                  -0.43388373911755812047576833284836,
                                  -0.97492791218182360701813168299393,
                                  -0.78183148246802980870844452667406};
};

template <typename T, int R>
struct DftOdd {
  __device__ __forceinline__ static void Run(Cx<T>* a) {
    constexpr int H = (R - 1) / 2;
    Cx<T> sp[H], sm[H];
#pragma unroll
    for (int j = 1; j <= H; ++j) {
      sp[j - 1] = Add(a[j], a[R - j]);
      sm[j - 1] = Sub(a[j], a[R - j]);
    }
    const Cx<T> a0 = a[0];
    Cx<T> y0 = a0;
#pragma unroll
    for (int j = 0; j < H; ++j) y0 = Add(y0, sp[j]);
#pragma unroll
    for (int k = 1; k <= H; ++k) {
      Cx<T> re = a0, im = {T(0), T(0)};
#pragma unroll
      for (int j = 1; j <= H; ++j) {
        const T cj = T(OddTables<R>::c[(j * k) % R]);
        const T sj = T(OddTables<R>::s[(j * k) % R]);
        re = {re.x + cj * sp[j - 1].x, re.y + cj * sp[j - 1].y};
        im = {im.x + sj * sm[j - 1].x, im.y + sj * sm[j - 1].y};
      }
      // y_k = re - i im, y_{R-k} = re + i im
      a[k] = {re.x + im.y, re.y - im.x};
      a[R - k] = {re.x - im.y, re.y + im.x};
    }
    a[0] = y0;
  }
};
template <typename T>
struct Dft<T, 3> : DftOdd<T, 3> {};
template <typename T>
struct Dft<T, 5> : DftOdd<T, 5> {};
template <typename T>
struct Dft<T, 7> : DftOdd<T, 7> {};

// composite radices R = P x Q (Cooley-Tukey in registers):
// X[k2 + Q k3] = sum_k1 W_P^{k1 k3} W_R^{k1 k2} sum_n2 x[k1 + P n2] W_Q^{n2 k2}
template <typename T, int P, int Q>
struct DftComposite {
  __device__ __forceinline__ static void Run(Cx<T>* a, const double (*w)[2]) {
    constexpr int R = P * Q;
    Cx<T> t[P][Q];
#pragma unroll
    for (int k1 = 0; k1 < P; ++k1) {
#pragma unroll
      for (int n2 = 0; n2 < Q; ++n2) t[k1][n2] = a[k1 + P * n2];
      Dft<T, Q>::Run(t[k1]);
#pragma unroll
      for (int k2 = 1; k2 < Q; ++k2)
        if (k1 > 0) {
          const int m = (k1 * k2) % R;
          t[k1][k2] = Mul(t[k1][k2], Cx<T>{T(w[m][0]), T(w[m][1])});
        }
    }
#pragma unroll
    for (int k2 = 0; k2 < Q; ++k2) {
      Cx<T> u[P];
#pragma unroll
      for (int k1 = 0; k1 < P; ++k1) u[k1] = t[k1][k2];
      Dft<T, P>::Run(u);
#pragma unroll
      for (int k3 = 0; k3 < P; ++k3) a[k2 + Q * k3] = u[k3];
    }
  }
};

// exp(-2 pi i m / 16), exp(-2 pi i m / 9)
__device__ constexpr double kW16[16][2] = {
    {1.0, 0.0},
    {0.92387953251128675612818318939679, -0.38268343236508977172845998403040},
    {0.70710678118654752440084436210485, -0.70710678118654752440084436210485},
    {0.38268343236508977172845998403040, -0.92387953251128675612818318939679},
    {0.0, -1.0},
    {-0.38268343236508977172845998403040, -0.92387953251128675612818318939679},
    {-0.70710678118654752440084436210485, -0.70710678118654752440084436210485},
    {-0.92387953251128675612818318939679, -0.38268343236508977172845998403040},
    {-1.0, 0.0},
    {-0.92387953251128675612818318939679, 0.38268343236508977172845998403040},
    {-0.70710678118654752440084436210485, 0.70710678118654752440084436210485},
    {-0.38268343236508977172845998403040, 0.92387953251128675612818318939679},
    {0.0, 1.0},
    {0.38268343236508977172845998403040, 0.92387953251128675612818318939679},
    {0.70710678118654752440084436210485, 0.70710678118654752440084436210485},
    {0.92387953251128675612818318939679, 0.38268343236508977172845998403040}};
__device__ constexpr double kW9[9][2] = {
    {1.0, 0.0},
    {0.76604444311897803520239265055542, -0.64278760968653932632264340990726},
    {0.17364817766693034885171662676931, -0.98480775301220805936674302458952},
    {-0.5, -0.86602540378443864676372317075294},
    {-0.93969262078590838405410927732473, -0.34202014332566873304409961468226},
    {-0.93969262078590838405410927732473, 0.34202014332566873304409961468226},
    {-0.5, 0.86602540378443864676372317075294},
    {0.17364817766693034885171662676931, 0.98480775301220805936674302458952},
    {0.76604444311897803520239265055542, 0.64278760968653932632264340990726}};

template <typename T>
struct Dft<T, 16> {
  __device__ __forceinline__ static void Run(Cx<T>* a) {
    DftComposite<T, 4, 4>::Run(a, kW16);
  }
};
template <typename T>
struct Dft<T, 9> {
  __device__ __forceinline__ static void Run(Cx<T>* a) {
    DftComposite<T, 3, 3>::Run(a, kW9);
  }
};
}  // namespace rdl
