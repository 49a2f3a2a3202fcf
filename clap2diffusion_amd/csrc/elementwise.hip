// Small HBM-bound kernels around the hot path: timestep embedding, fused
// CFG + DDIM update, latent layout conversion, HTSAT input stage (BatchNorm +
// bicubic resize + mel->image fold + 4x4 patch cut), Swin patch-merge gather,
// token mean pool and L2 normalisation.
#include "common.h"
#include <math.h>

namespace c2d {

__global__ void timestep_emb_kernel(const float* t_table, const int* step_index, int n, int dim, f16* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int half = dim / 2;
    if (i >= n * half) return;
    const int j = i % half, row = i / half;
    const float t = t_table[step_index ? *step_index : 0];
    // diffusers get_timestep_embedding: exp(-ln(1e4) * j / half), fp32
    const float f = expf(-9.210340371976184f * (float)j / (float)half);
    const float a = t * f;
    out[(size_t)row * dim + j] = (f16)cosf(a);
    out[(size_t)row * dim + half + j] = (f16)sinf(a);
}

__global__ void cfg_ddim_kernel(const f16* eps, float* x, int b, int c, int hw, float gsc, const float* coef,
                                const int* step_index) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= b * c * hw) return;
    const int p = i % hw, ch = (i / hw) % c, bi = i / (hw * c);
    const int st = *step_index;
    const float a_t = coef[st * 2], a_p = coef[st * 2 + 1];
    const float eu = (float)eps[((size_t)bi * hw + p) * c + ch];
    const float ec = (float)eps[((size_t)(b + bi) * hw + p) * c + ch];
    const float e = eu + gsc * (ec - eu);
    const float xv = x[i];
    const float x0 = (xv - sqrtf(1.0f - a_t) * e) / sqrtf(a_t);
    x[i] = sqrtf(a_p) * x0 + sqrtf(1.0f - a_p) * e;
}

__global__ void step_advance_kernel(int* step_index) { *step_index += 1; }

__global__ void latent_to_nhwc_kernel(const float* x, int n, int c, int hw, int cpad, int dup, f16* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n * hw * cpad) return;
    const int ch = i % cpad, p = (i / cpad) % hw, bi = i / (cpad * hw);
    const float v = ch < c ? x[((size_t)bi * c + ch) * hw + p] : 0.f;
    out[i] = (f16)v;
    if (dup) out[(size_t)n * hw * cpad + i] = (f16)v;
}

__global__ void add_kernel(const f16x8* a, const f16x8* b, f16x8* o, size_t n8) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i < n8; i += (size_t)gridDim.x * blockDim.x) o[i] = a[i] + b[i];
}

// torch upsample_bicubic2d cubic convolution, A = -0.75
__device__ __forceinline__ float cc1(float x) { const float A = -0.75f; return ((A + 2.f) * x - (A + 3.f)) * x * x + 1.f; }
__device__ __forceinline__ float cc2(float x) { const float A = -0.75f; return ((A * x - 5.f * A) * x + 8.f * A) * x - 4.f * A; }

__global__ void mel_patches_kernel(const float* mel, int b, int T, const float* bn_scale, const float* bn_shift, f16* out) {
    // out [b*4096][64]: token (py, px), column k = dy*4 + dx (16 used)
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= b * 4096 * 64) return;
    const int col = i & 63, tok = (i >> 6) & 4095, bi = i >> 18;
    float val = 0.f;
    if (col < 16) {
        const int dy = col >> 2, dx = col & 3;
        const int py = tok >> 6, px = tok & 63;
        const int r = 4 * py + dy, cidx = 4 * px + dx;      // image row / col in 256x256
        const int tt = (r >> 6) * 256 + cidx;                // time index in [0, 1024)
        const int f = r & 63;                                // mel bin
        const float* m = mel + (size_t)bi * T * 64;
        const float sc = bn_scale[f], sh = bn_shift[f];
        if (T == 1024) {
            val = m[(size_t)tt * 64 + f] * sc + sh;
        } else {
            const float scale = (float)(T - 1) / 1023.f;     // align_corners = True
            const float real = scale * (float)tt;
            const int i0 = (int)floorf(real);
            const float u = real - (float)i0;
            const float w0 = cc2(u + 1.f), w1 = cc1(u), w2 = cc1(1.f - u), w3 = cc2(2.f - u);
            float acc = 0.f;
            const float ws[4] = {w0, w1, w2, w3};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                int idx = min(max(i0 - 1 + q, 0), T - 1);
                acc += ws[q] * (m[(size_t)idx * 64 + f] * sc + sh);
            }
            val = acc;
        }
    }
    out[i] = (f16)val;
}

__global__ void patch_merge_kernel(const f16* x, int b, int h, int w, int c, f16* out) {
    // one thread per 8-channel chunk of an output token: out [b][h/2*w/2][4c]
    const int nch = c >> 3;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int h2 = h / 2, w2 = w / 2;
    const size_t total = (size_t)b * h2 * w2 * 4 * nch;
    if (i >= total) return;
    const int ch = i % nch;
    const int part = (i / nch) % 4;
    const size_t tok = i / (4 * nch);
    const int bi = tok / (h2 * w2), r = tok % (h2 * w2);
    const int oy = r / w2, ox = r % w2;
    // torch.cat([x[:, row::2, col::2] for col in range(2) for row in range(2)])
    const int col = part >> 1, row = part & 1;
    const int iy = 2 * oy + row, ix = 2 * ox + col;
    const f16x8 v = *reinterpret_cast<const f16x8*>(x + (((size_t)bi * h + iy) * w + ix) * c + ch * 8);
    *reinterpret_cast<f16x8*>(out + tok * 4 * c + part * c + ch * 8) = v;
}

__global__ void row_mean_kernel(const f16* x, int b, int rows, int c, int ld, float* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= b * c) return;
    const int bi = i / c, ch = i % c;
    float s = 0.f;
    for (int r = 0; r < rows; ++r) s += (float)x[((size_t)bi * rows + r) * ld + ch];
    out[i] = s / (float)rows;
}

__global__ void l2norm_kernel(float* x, int m, int c) {
    const int row = blockIdx.x;
    __shared__ float part[4];
    float s = 0.f;
    for (int j = threadIdx.x; j < c; j += blockDim.x) s += x[(size_t)row * c + j] * x[(size_t)row * c + j];
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
    __syncthreads();
    float tot = 0.f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) tot += part[i];
    const float inv = 1.0f / fmaxf(sqrtf(tot), 1e-12f);
    for (int j = threadIdx.x; j < c; j += blockDim.x) x[(size_t)row * c + j] *= inv;
}

// Row softmax for the materialised single-head attention of the VAE mid block
// (diffusers Attention with one 512-wide head: softmax(Q K^T / sqrt(d)) over 4096 /
// 9216 keys; the 1/sqrt(d) is folded into to_q).  One 256-thread workgroup per row,
// the row held in registers (NCH 16-B chunks per thread): fp32 max, exp2, sum, scale,
// fp16 out -- one HBM read and one write per score.
template <int NCH>
__global__ void __launch_bounds__(256) softmax_rows_kernel(const f16* x, int cols, int ld, f16* out, int ldo) {
    const size_t row = blockIdx.x;
    const int tid = threadIdx.x;
    __shared__ float part[4];
    f16x8 v[NCH];
    float mx = -INFINITY;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
        const int c0 = (i * 256 + tid) * 8;
        if (c0 < cols) {
            v[i] = *reinterpret_cast<const f16x8*>(x + row * ld + c0);
#pragma unroll
            for (int j = 0; j < 8; ++j) mx = fmaxf(mx, (float)v[i][j]);
        }
    }
    mx = wave_max(mx);
    if ((tid & 63) == 0) part[tid >> 6] = mx;
    __syncthreads();
    mx = fmaxf(fmaxf(part[0], part[1]), fmaxf(part[2], part[3]));
    __syncthreads();
    const float L2E = 1.4426950408889634f, ml = mx * L2E;
    float e[NCH][8];
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
        const int c0 = (i * 256 + tid) * 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            e[i][j] = c0 < cols ? __builtin_amdgcn_exp2f(fmaf((float)v[i][j], L2E, -ml)) : 0.f;
            sum += e[i][j];
        }
    }
    sum = wave_sum(sum);
    if ((tid & 63) == 0) part[tid >> 6] = sum;
    __syncthreads();
    const float inv = 1.0f / (part[0] + part[1] + part[2] + part[3]);
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
        const int c0 = (i * 256 + tid) * 8;
        if (c0 < cols) {
            f16x8 o;
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = (f16)(e[i][j] * inv);
            *reinterpret_cast<f16x8*>(out + row * ldo + c0) = o;
        }
    }
}

// Weight prepack: fp32 [cout][cin][k][k] (PyTorch
// conv / linear layout, k = 1 for a linear) -> fp16 [cout][kpad], K ordered
// (ky, kx, channel) over cin_pad channels (channels >= cin and K >= k*k*cin_pad are 0).
__global__ void pack_weights_kernel(const float* __restrict__ w, int cout, int cin, int ksz, int cin_pad, int kpad,
                                    f16* __restrict__ out) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)cout * kpad) return;
    const int o = (int)(i / kpad), kk = (int)(i - (size_t)o * kpad);
    float v = 0.f;
    if (kk < ksz * ksz * cin_pad) {
        const int tap = kk / cin_pad, c = kk - tap * cin_pad;
        const int ky = tap / ksz, kx = tap - ky * ksz;
        if (c < cin) v = w[(((size_t)o * cin + c) * ksz + ky) * ksz + kx];
    }
    out[i] = (f16)v;
}

}  // namespace c2d

using namespace c2d;

extern "C" const char* c2d_version(void) { return "c2d_hip gfx950 r6"; }

extern "C" int c2d_timestep_embedding(const float* t_table, const int* step_index, int n, int dim, void* out,
                                      void* stream) {
    if (!t_table || !out) return C2D_E_ARG;
    if (dim & 1 || n <= 0) return C2D_E_SHAPE;
    const int tot = n * dim / 2;
    hipLaunchKernelGGL(timestep_emb_kernel, dim3((tot + 255) / 256), dim3(256), 0, (hipStream_t)stream, t_table,
                       step_index, n, dim, (f16*)out);
    return check_launch();
}

extern "C" int c2d_cfg_ddim_step(const void* eps, float* x, int b, int c, int hw, float guidance, const float* coef,
                                 int* step_index, int advance, void* stream) {
    if (!eps || !x || !coef || !step_index) return C2D_E_ARG;
    if (b <= 0 || c <= 0 || hw <= 0) return C2D_E_SHAPE;
    const int tot = b * c * hw;
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(cfg_ddim_kernel, dim3((tot + 255) / 256), dim3(256), 0, s, (const f16*)eps, x, b, c, hw,
                       guidance, coef, step_index);
    if (advance) hipLaunchKernelGGL(step_advance_kernel, dim3(1), dim3(1), 0, s, step_index);
    return check_launch();
}

extern "C" int c2d_latent_to_nhwc(const float* x, int n, int c, int hw, int cpad, int dup, void* out, void* stream) {
    if (!x || !out) return C2D_E_ARG;
    if (cpad < c || n <= 0) return C2D_E_SHAPE;
    const int tot = n * hw * cpad;
    hipLaunchKernelGGL(latent_to_nhwc_kernel, dim3((tot + 255) / 256), dim3(256), 0, (hipStream_t)stream, x, n, c,
                       hw, cpad, dup, (f16*)out);
    return check_launch();
}

__global__ void upsample2x_kernel(const f16x8* __restrict__ x, int h, int w, int c8, f16x8* __restrict__ out,
                                  size_t total) {
    // one thread per output 16-byte chunk; consecutive threads walk channels then columns
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const int cc = (int)(i % c8);
        const size_t pix = i / c8;
        const int ox = (int)(pix % (2 * w));
        const size_t r = pix / (2 * w);
        const int oy = (int)(r % (2 * h));
        const size_t n = r / (2 * h);
        out[i] = x[((n * h + (oy >> 1)) * w + (ox >> 1)) * c8 + cc];
    }
}

extern "C" int c2d_upsample_nearest2x(const void* x, int n, int h, int w, int c, void* out, void* stream) {
    if (!x || !out) return C2D_E_ARG;
    if (n <= 0 || h <= 0 || w <= 0 || c <= 0 || (c & 7)) return C2D_E_SHAPE;
    if (!aligned16(x) || !aligned16(out)) return C2D_E_ALIGN;
    const size_t total = (size_t)n * 4 * h * w * (c / 8);
    const unsigned blocks = (unsigned)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192);
    hipLaunchKernelGGL(upsample2x_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const f16x8*)x, h, w, c / 8,
                       (f16x8*)out, total);
    return check_launch();
}

extern "C" int c2d_add(const void* a, const void* b, void* out, size_t n, void* stream) {
    if (!a || !b || !out) return C2D_E_ARG;
    if (n & 7) return C2D_E_SHAPE;
    if (!aligned16(a) || !aligned16(b) || !aligned16(out)) return C2D_E_ALIGN;
    const size_t n8 = n / 8;
    const unsigned blocks = (unsigned)((n8 + 255) / 256 < 4096 ? (n8 + 255) / 256 : 4096);
    if (!n8) return C2D_OK;
    hipLaunchKernelGGL(add_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const f16x8*)a, (const f16x8*)b,
                       (f16x8*)out, n8);
    return check_launch();
}

extern "C" int c2d_htsat_mel_patches(const float* mel, int b, int t, const float* bn_scale, const float* bn_shift,
                                     void* out, void* stream) {
    if (!mel || !bn_scale || !bn_shift || !out) return C2D_E_ARG;
    if (b <= 0 || t < 2 || t > 1024) return C2D_E_SHAPE;
    const int tot = b * 4096 * 64;
    hipLaunchKernelGGL(mel_patches_kernel, dim3((tot + 255) / 256), dim3(256), 0, (hipStream_t)stream, mel, b, t,
                       bn_scale, bn_shift, (f16*)out);
    return check_launch();
}

extern "C" int c2d_patch_merge_gather(const void* x, int b, int h, int w, int c, void* out, void* stream) {
    if (!x || !out) return C2D_E_ARG;
    if ((h & 1) || (w & 1) || (c & 7)) return C2D_E_SHAPE;
    if (!aligned16(x) || !aligned16(out)) return C2D_E_ALIGN;
    const size_t tot = (size_t)b * (h / 2) * (w / 2) * 4 * (c / 8);
    hipLaunchKernelGGL(patch_merge_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       (const f16*)x, b, h, w, c, (f16*)out);
    return check_launch();
}

extern "C" int c2d_row_mean(const void* x, int b, int rows, int c, int ld, float* out, void* stream) {
    if (!x || !out) return C2D_E_ARG;
    const int tot = b * c;
    hipLaunchKernelGGL(row_mean_kernel, dim3((tot + 255) / 256), dim3(256), 0, (hipStream_t)stream, (const f16*)x, b,
                       rows, c, ld, out);
    return check_launch();
}

extern "C" int c2d_l2_normalize(float* x, int m, int c, void* stream) {
    if (!x) return C2D_E_ARG;
    hipLaunchKernelGGL(l2norm_kernel, dim3(m), dim3(256), 0, (hipStream_t)stream, x, m, c);
    return check_launch();
}

extern "C" int c2d_softmax_rows(const void* x, int rows, int cols, int ld, void* out, int ldo, void* stream) {
    if (!x || !out) return C2D_E_ARG;
    if (rows < 0 || cols <= 0 || cols % 8 || cols > 16384 || ld < cols || ldo < cols) return C2D_E_SHAPE;
    if (((uintptr_t)x | (uintptr_t)out) & 15 || ld % 8 || ldo % 8) return C2D_E_ALIGN;
    if (rows == 0) return 0;
    const int nch = (cols / 8 + 255) / 256;
    const hipStream_t s = (hipStream_t)stream;
#define C2D_SM(N) hipLaunchKernelGGL(softmax_rows_kernel<N>, dim3(rows), dim3(256), 0, s, (const f16*)x, cols, ld, (f16*)out, ldo)
    if (nch <= 1) C2D_SM(1);
    else if (nch <= 2) C2D_SM(2);
    else if (nch <= 4) C2D_SM(4);
    else C2D_SM(8);
#undef C2D_SM
    return check_launch();
}

extern "C" int c2d_pack_weights(const float* w, int cout, int cin, int ksize, int cin_pad, int kpad, void* out,
                                void* stream) {
    if (!w || !out) return C2D_E_ARG;
    if (cout <= 0 || cin <= 0 || (ksize != 1 && ksize != 3) || cin_pad < cin || kpad % 64 ||
        kpad < ksize * ksize * cin_pad)
        return C2D_E_SHAPE;
    const size_t n = (size_t)cout * kpad;
    hipLaunchKernelGGL(pack_weights_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, w,
                       cout, cin, ksize, cin_pad, kpad, (f16*)out);
    return check_launch();
}
