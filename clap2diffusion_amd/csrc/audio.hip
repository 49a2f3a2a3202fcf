// CLAP log-mel front end for gfx950: the reference's audio composition
// CLAPAudioEncoder.preprocess_audio (models/audio_encoder.py:121-129: zero-pad to
// target_length * sample_rate = max_len samples, or keep the first max_len) followed
// by transformers' ClapFeatureExtractor on that exactly-max_len clip
// (feature_extraction_clap.py _get_input_mel: neither the repeat-pad nor the random
// crop fires at exact length; _np_extract_fbank_features, audio_utils.spectrogram /
// power_to_db), called by the reference at models/audio_encoder.py:163-171.
//
// One 256-thread workgroup per (clip, frame):
//   1. gather the frame's 1024 samples: the clip zero-padded / truncated to max_len
//      (lengths are clamped to [0, max_len], so a longer clip keeps its first max_len
//      samples and an empty one reads as silence), then the centre reflect pad of
//      n_fft/2 (np.pad mode "reflect"), times the periodic Hann window;
//   2. 1024-point complex FFT in LDS, radix-2 Stockham (natural-order output, fp32,
//      twiddles from sincospi) -- fp32 keeps bins ~120 dB below the frame peak exact,
//      which an fp16 DFT-as-GEMM would not (the dB features feed a BatchNorm);
//   3. |X_k|^2 for the 513 one-sided bins, the Slaney mel filter dot products over
//      each filter's non-zero bin range, max(., 1e-10), 10 log10.
// Output fp32 [b][frames][n_mels], frame-major so the mel row is one coalesced store.
#include "common.h"
#include <math.h>

namespace c2d {

constexpr int MEL_NFFT = 1024;
constexpr int MEL_NBIN = MEL_NFFT / 2 + 1;

__global__ void __launch_bounds__(256) clap_log_mel_kernel(const float* __restrict__ wave,
                                                           const long long* __restrict__ offsets,
                                                           const int* __restrict__ lengths, int max_len, int hop,
                                                           int frames, const float* __restrict__ window,
                                                           const float* __restrict__ filt,
                                                           const int* __restrict__ frange, int n_mels,
                                                           float* __restrict__ out) {
    __shared__ float2 buf[2][MEL_NFFT];
    __shared__ float pw[MEL_NBIN + 3];
    const int tid = threadIdx.x;
    const int fr = blockIdx.x % frames, bi = blockIdx.x / frames;
    const float* x = wave + offsets[bi];
    const int n = min(max(lengths[bi], 0), max_len);   // zero-pad / truncate (audio_encoder.py:123-129)

#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = tid + 256 * r;
        int p = fr * hop + i - MEL_NFFT / 2;   // position in the zero-padded clip
        if (p < 0) p = -p;                     // reflect (edge sample not repeated)
        if (p >= max_len) p = 2 * (max_len - 1) - p;
        const float s = p < n ? x[p] : 0.f;
        buf[0][i] = make_float2(s * window[i], 0.f);
    }
    __syncthreads();

    // Stockham radix-2: stage with half-length ns reads j and j + N/2, writes
    // (j / ns) * 2 ns + j % ns and that + ns
    int src = 0;
    for (int ns = 1; ns < MEL_NFFT; ns <<= 1) {
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const int j = tid + 256 * r;
            const int k = j & (ns - 1);
            const float2 a0 = buf[src][j], a1 = buf[src][j + MEL_NFFT / 2];
            float sn, cs;
            sincospif(-(float)k / (float)ns, &sn, &cs);
            const float2 t = make_float2(a1.x * cs - a1.y * sn, a1.x * sn + a1.y * cs);
            const int o = ((j - k) << 1) + k;
            buf[src ^ 1][o] = make_float2(a0.x + t.x, a0.y + t.y);
            buf[src ^ 1][o + ns] = make_float2(a0.x - t.x, a0.y - t.y);
        }
        src ^= 1;
        __syncthreads();
    }

    for (int k = tid; k < MEL_NBIN; k += 256) {
        const float2 v = buf[src][k];
        pw[k] = v.x * v.x + v.y * v.y;
    }
    __syncthreads();

    for (int m = tid; m < n_mels; m += 256) {
        const float* fm = filt + (size_t)m * MEL_NBIN;
        float acc = 0.f;
        for (int k = frange[2 * m]; k < frange[2 * m + 1]; ++k) acc = fmaf(fm[k], pw[k], acc);
        out[((size_t)bi * frames + fr) * n_mels + m] = 10.f * log10f(fmaxf(acc, 1e-10f));
    }
}

}  // namespace c2d

using namespace c2d;

extern "C" int c2d_clap_log_mel(const float* wave, const long long* offsets, const int* lengths, int b, int max_len,
                                int n_fft, int hop, const float* window, const float* mel_filters,
                                const int* filter_range, int n_mels, float* out, void* stream) {
    if (!wave || !offsets || !lengths || !window || !mel_filters || !filter_range || !out) return C2D_E_ARG;
    if (n_fft != MEL_NFFT || hop <= 0 || max_len <= MEL_NFFT / 2 || n_mels <= 0 || b < 0) return C2D_E_SHAPE;
    if (b == 0) return 0;
    const int frames = 1 + max_len / hop;   // centre-padded length max_len + n_fft, minus n_fft, over hop
    hipLaunchKernelGGL(clap_log_mel_kernel, dim3(b * frames), dim3(256), 0, (hipStream_t)stream, wave, offsets,
                       lengths, max_len, hop, frames, window, mel_filters, filter_range, n_mels, out);
    return check_launch();
}
