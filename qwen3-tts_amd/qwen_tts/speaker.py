"""Speaker encoder (mel + ECAPA-TDNN x-vector) on the MI355X kernels (voice-clone front end).

Replaces `Qwen3TTSForConditionalGeneration.extract_speaker_embedding` (M = qwen_tts/core/models/
modeling_qwen3_tts.py:1940-1954): `mel_spectrogram` (M:405-470) + `Qwen3TTSSpeakerEncoder` (M:325-398).

* STFT as an MFMA GEMM: the reflect-padded waveform is viewed as [rows][hop] (hop = 256) and every frame
  (n_fft = 1024 = 4 hops) is a 4-tap implicit conv over that view; the periodic Hann window is folded into the
  [2*513][1024] cos/sin basis, so one fp32 GEMM emits the (re, im) pairs of all frames.  qt_mel_logmag then
  forms sqrt(re^2 + im^2 + 1e-9), applies the slaney mel filterbank and the log clamp.
* ECAPA: every Conv1d is the weight-tiled GEMM (ReLU / sigmoid / tanh∘ReLU fused in the epilogue); the
  reflect "same" padding is a qt_pad_time pass (fused with the Res2Net running sum); squeeze-excitation and
  attentive statistics pooling are qt_time_stats + two M = B GEMVs + qt_scale_add.  Block outputs are written
  straight into the multi-layer-aggregation buffer and the pooling's [h | mean | std] buffer (no concat pass).
"""
from __future__ import annotations

from typing import Dict

import numpy as np
import torch

from . import _hip
from . import kernels as K


def _hz_to_mel(f):
    f = np.asanyarray(f, dtype=np.float64)
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, np.log(6.4) / 27.0
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-300) / min_log_hz) / logstep, f / f_sp)


def _mel_to_hz(m):
    m = np.asanyarray(m, dtype=np.float64)
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, np.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), f_sp * m)


def mel_filterbank(sr: int, n_fft: int, n_mels: int, fmin: float, fmax: float) -> np.ndarray:
    """The slaney-normalised mel filterbank of librosa.filters.mel(htk=False, norm="slaney") (M:435-437; librosa's
    published algorithm: slaney mel scale, triangular ramps over the rfft bin frequencies, area normalisation),
    float32 [n_mels][1 + n_fft/2].  Computed once at load time on the host."""
    w = np.zeros((n_mels, 1 + n_fft // 2), dtype=np.float32)
    fft_f = np.fft.rfftfreq(n=n_fft, d=1.0 / sr)
    mel_f = _mel_to_hz(np.linspace(_hz_to_mel(fmin), _hz_to_mel(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fft_f)
    for i in range(n_mels):
        w[i] = np.maximum(0, np.minimum(-ramps[i] / fdiff[i], ramps[i + 2] / fdiff[i + 1]))
    w *= (2.0 / (mel_f[2: n_mels + 2] - mel_f[:n_mels]))[:, np.newaxis]
    return w


def speaker_config(cfg: dict) -> dict:
    c = dict(mel_dim=128, enc_dim=1024, enc_channels=[512, 512, 512, 512, 1536], enc_kernel_sizes=[5, 3, 3, 3, 1],
             enc_dilations=[1, 2, 3, 4, 1], enc_attention_channels=128, enc_res2net_scale=8, enc_se_channels=128,
             sample_rate=24000)
    c.update(cfg.get("speaker_encoder_config", {}) or {})
    return c


def speaker_specs(cfg: dict):
    """(name, shape) of the speaker encoder parameters in model.safetensors (prefix `speaker_encoder.`, M:1823)."""
    c = speaker_config(cfg)
    ch, ks, sc, se = c["enc_channels"], c["enc_kernel_sizes"], c["enc_res2net_scale"], c["enc_se_channels"]
    p = "speaker_encoder"
    s = [(f"{p}.blocks.0.conv.weight", (ch[0], c["mel_dim"], ks[0])), (f"{p}.blocks.0.conv.bias", (ch[0],))]
    for i in range(1, len(ch) - 1):
        q, cin, co = f"{p}.blocks.{i}", ch[i - 1], ch[i]
        s += [(f"{q}.tdnn1.conv.weight", (co, cin, 1)), (f"{q}.tdnn1.conv.bias", (co,))]
        for j in range(sc - 1):
            s += [(f"{q}.res2net_block.blocks.{j}.conv.weight", (co // sc, cin // sc, ks[i])),
                  (f"{q}.res2net_block.blocks.{j}.conv.bias", (co // sc,))]
        s += [(f"{q}.tdnn2.conv.weight", (co, co, 1)), (f"{q}.tdnn2.conv.bias", (co,)),
              (f"{q}.se_block.conv1.weight", (se, co, 1)), (f"{q}.se_block.conv1.bias", (se,)),
              (f"{q}.se_block.conv2.weight", (co, se, 1)), (f"{q}.se_block.conv2.bias", (co,))]
    cm, ac = ch[-1], c["enc_attention_channels"]
    s += [(f"{p}.mfa.conv.weight", (cm, sum(ch[1:-1]), ks[-1])), (f"{p}.mfa.conv.bias", (cm,)),
          (f"{p}.asp.tdnn.conv.weight", (ac, cm * 3, 1)), (f"{p}.asp.tdnn.conv.bias", (ac,)),
          (f"{p}.asp.conv.weight", (cm, ac, 1)), (f"{p}.asp.conv.bias", (cm,)),
          (f"{p}.fc.weight", (c["enc_dim"], cm * 2, 1)), (f"{p}.fc.bias", (c["enc_dim"],))]
    return s


class SpeakerEncoder:
    N_FFT, HOP, WIN, N_MELS, FMIN, FMAX, SR = 1024, 256, 1024, 128, 0, 12000, 24000  # M:1943-1951

    def __init__(self, cfg: dict, weights: Dict[str, torch.Tensor], dtype="bf16", device="cuda"):
        _hip.lib()
        self.c = c = speaker_config(cfg)
        self.dev = dev = torch.device(device)
        self.wdt = wdt = torch.bfloat16 if dtype == "bf16" else torch.float32
        g = lambda n: (weights[n] if isinstance(weights[n], torch.Tensor) else torch.from_numpy(weights[n])).to(dev).float()  # noqa: E731
        ch, ks, dl = c["enc_channels"], c["enc_kernel_sizes"], c["enc_dilations"]
        if len(ch) != len(ks) or len(ch) != len(dl):
            raise ValueError("enc_channels, enc_kernel_sizes and enc_dilations should have same length")
        if c["mel_dim"] != self.N_MELS or ks[-1] != 1:
            raise NotImplementedError("speaker encoder needs 128 mels and a 1x1 aggregation conv")
        # mel front end: DFT basis with the periodic Hann window folded in (fp32: magnitudes feed a log)
        n, nb = self.N_FFT, self.N_FFT // 2 + 1
        s = np.arange(n, dtype=np.float64)
        win = 0.5 - 0.5 * np.cos(2 * np.pi * s / self.WIN)
        ang = 2 * np.pi * np.outer(np.arange(nb), s) / n
        basis = np.empty((2 * nb, n), dtype=np.float64)
        basis[0::2] = win * np.cos(ang)
        basis[1::2] = -win * np.sin(ang)
        taps = n // self.HOP
        w3 = torch.from_numpy(basis.astype(np.float32)).to(dev).reshape(2 * nb, taps, self.HOP)
        self.dft = K.tile(w3.reshape(2 * nb, taps * self.HOP), torch.float32, taps=taps, cin=self.HOP, cin_pad=self.HOP,
                          K=taps * self.HOP)
        self.dft.dil = 1
        self.nbin = nb
        self.mel_basis = torch.from_numpy(mel_filterbank(self.SR, n, self.N_MELS, self.FMIN, self.FMAX)).to(dev).contiguous()
        # ECAPA
        p = "speaker_encoder"
        conv = lambda q, d=1: K.tile_conv(g(f"{q}.weight"), g(f"{q}.bias"), wdt, d)  # noqa: E731
        lin = lambda q: K.tile_linear(g(f"{q}.weight")[:, :, 0], wdt, g(f"{q}.bias"))  # noqa: E731
        self.b0 = dict(w=conv(f"{p}.blocks.0.conv", dl[0]), k=ks[0], d=dl[0])
        self.sc = c["enc_res2net_scale"]
        self.blocks = []
        for i in range(1, len(ch) - 1):
            q = f"{p}.blocks.{i}"
            self.blocks.append(dict(
                C=ch[i], k=ks[i], d=dl[i], tdnn1=lin(f"{q}.tdnn1.conv"), tdnn2=lin(f"{q}.tdnn2.conv"),
                res2=[conv(f"{q}.res2net_block.blocks.{j}.conv", dl[i]) for j in range(self.sc - 1)],
                se1=lin(f"{q}.se_block.conv1"), se2=lin(f"{q}.se_block.conv2")))
            if ch[i] != ch[i - 1]:
                raise NotImplementedError("SE-Res2Net blocks with a channel change (no residual projection)")
        self.C_mfa = sum(ch[1:-1])
        self.mfa = lin(f"{p}.mfa.conv")
        self.cm = ch[-1]
        self.asp_tdnn = lin(f"{p}.asp.tdnn.conv")
        self.asp_conv = lin(f"{p}.asp.conv")
        self.fc = lin(f"{p}.fc")
        K.gemm_workspace(dev)
        torch.cuda.synchronize(dev)

    # ------------------------------------------------------------------------------------------------
    def mel(self, wav: torch.Tensor, check_range: bool = True) -> torch.Tensor:
        """mel_spectrogram (M:405-470) of one fp32 device waveform [L] -> log-mel [frames][128] (time-major)."""
        L = int(wav.shape[0])
        pad = (self.N_FFT - self.HOP) // 2
        if L <= pad:
            raise ValueError(f"reference audio too short for the speaker encoder ({L} samples; reflect padding "
                             f"needs more than {pad})")
        if check_range:
            self._warn_range([wav])
        Lp = L + 2 * pad
        F_ = (Lp - self.N_FFT) // self.HOP + 1
        rows = -(-Lp // self.HOP)
        y = torch.empty(rows * self.HOP, dtype=torch.float32, device=self.dev)
        K.pad_time(wav.contiguous().float(), 1, L, 1, pad, pad, _hip.PAD_REFLECT, y, t_total=rows * self.HOP)
        spec = torch.empty(F_, 2 * self.nbin, dtype=torch.float32, device=self.dev)
        K.gemm(y, self.dft, spec, F_, self.HOP, 2 * self.nbin, conv=(rows, F_, 0, 1))
        out = torch.empty(F_, self.N_MELS, dtype=torch.float32, device=self.dev)
        K.mel_logmag(spec, 2 * self.nbin, F_, self.nbin, self.mel_basis, self.N_MELS, out)
        return out

    def _tdnn(self, x, W, B, T, cin, k, d, out, ldx=None, ldo=None, x2=None, ldx2=None):
        """TimeDelayNetBlock (M:246-266): reflect "same" pad (+ optional running sum x2) then conv + ReLU."""
        tot = d * (k - 1)
        if tot == 0:
            K.gemm(x, W, out, B * T, ldx or cin, ldo or W.N, act=_hip.ACT_RELU)
            return
        l, r = tot // 2, tot - tot // 2
        xp = torch.empty(B * (T + tot), cin, dtype=torch.float32, device=self.dev)
        K.pad_time(x, B, T, cin, l, r, _hip.PAD_REFLECT, xp, x2=x2, ldx=ldx or cin, ldx2=ldx2)
        K.gemm(xp, W, out, B * T, cin, ldo or W.N, conv=(T + tot, T, 0, d), act=_hip.ACT_RELU)

    def forward(self, mels: torch.Tensor) -> torch.Tensor:
        """Qwen3TTSSpeakerEncoder.forward (M:378-398): log-mels fp32 [B][T][128] -> x-vectors fp32 [B][enc_dim]."""
        B, T, nm = mels.shape
        dev = self.dev
        mels = mels.contiguous()
        C0 = self.b0["w"].N
        h = torch.empty(B * T, C0, dtype=torch.float32, device=dev)
        self._tdnn(mels, self.b0["w"], B, T, nm, self.b0["k"], self.b0["d"], h)
        mfa_in = torch.empty(B * T, self.C_mfa, dtype=torch.float32, device=dev)
        prev, prev_ld, off = h, C0, 0
        for blk in self.blocks:
            C, sc = blk["C"], self.sc
            w = C // sc
            r2 = torch.empty(B * T, C, dtype=torch.float32, device=dev)
            K.gemm(prev, blk["tdnn1"], r2, B * T, prev_ld, C, act=_hip.ACT_RELU)
            for j in range(1, sc):  # Res2NetBlock (M:114-121): chunk j (+ output j-1 for j >= 2) -> tdnn
                self._tdnn(r2[:, j * w:], blk["res2"][j - 1], B, T, w, blk["k"], blk["d"], r2[:, j * w:], ldx=C, ldo=C,
                           x2=r2[:, (j - 1) * w:] if j >= 2 else None, ldx2=C)
            x2 = torch.empty(B * T, C, dtype=torch.float32, device=dev)
            K.gemm(r2, blk["tdnn2"], x2, B * T, C, C, act=_hip.ACT_RELU)
            se = torch.empty(B, C, dtype=torch.float32, device=dev)  # SqueezeExcitationBlock (M:143-151)
            K.time_stats(x2, B, T, C, se)
            s1 = torch.empty(B, blk["se1"].N, dtype=torch.float32, device=dev)
            K.gemm(se, blk["se1"], s1, B, C, blk["se1"].N, act=_hip.ACT_RELU)
            s2 = torch.empty(B, C, dtype=torch.float32, device=dev)
            K.gemm(s1, blk["se2"], s2, B, blk["se1"].N, C, act=_hip.ACT_SIGMOID)
            K.scale_add(x2, s2, prev, B, T, C, mfa_in[:, off:], ldr=prev_ld, ldo=self.C_mfa)
            prev, prev_ld = mfa_in[:, off:], self.C_mfa
            off += C
        cm = self.cm
        asp_in = torch.empty(B * T, 3 * cm, dtype=torch.float32, device=dev)  # [h | mean | std] (M:221-228)
        K.gemm(mfa_in, self.mfa, asp_in, B * T, self.C_mfa, 3 * cm, act=_hip.ACT_RELU)
        ms = torch.empty(B, 2 * cm, dtype=torch.float32, device=dev)
        K.time_stats(asp_in, B, T, cm, ms, ms[:, cm:], ldx=3 * cm, ld_out=2 * cm)
        K.bcast_rows(ms, B, T, 2 * cm, asp_in[:, cm:], ldv=2 * cm, ldo=3 * cm)
        a1 = torch.empty(B * T, self.asp_tdnn.N, dtype=torch.float32, device=dev)
        K.gemm(asp_in, self.asp_tdnn, a1, B * T, 3 * cm, self.asp_tdnn.N, act=_hip.ACT_RELU_TANH)
        lg = torch.empty(B * T, cm, dtype=torch.float32, device=dev)
        K.gemm(a1, self.asp_conv, lg, B * T, self.asp_tdnn.N, cm)
        pooled = torch.empty(B, 2 * cm, dtype=torch.float32, device=dev)
        K.time_stats(asp_in, B, T, cm, pooled, pooled[:, cm:], logits=lg, ldx=3 * cm, ldl=cm, ld_out=2 * cm)
        emb = torch.empty(B, self.fc.N, dtype=torch.float32, device=dev)
        K.gemm(pooled, self.fc, emb, B, 2 * cm, self.fc.N)
        return emb

    @staticmethod
    def _warn_range(wavs):
        """mel_spectrogram's range warnings (M:420-423), one host read for all clips."""
        mm = torch.stack([torch.stack(torch.aminmax(w)) for w in wavs]).cpu()
        for lo, hi in mm.tolist():
            if lo < -1.0:
                print(f"[WARNING] Min value of input waveform signal is {lo}")
            if hi > 1.0:
                print(f"[WARNING] Max value of input waveform signal is {hi}")

    def _dev_wav(self, wav) -> torch.Tensor:
        w = torch.as_tensor(np.asarray(wav, dtype=np.float32) if not isinstance(wav, torch.Tensor) else wav)
        return w.to(self.dev, torch.float32).reshape(-1)

    def embed(self, wav) -> torch.Tensor:
        """extract_speaker_embedding (M:1940-1954): 24 kHz mono waveform -> x-vector fp32 [enc_dim] (device)."""
        return self.forward(self.mel(self._dev_wav(wav))[None])[0]

    def embed_many(self, wavs) -> torch.Tensor:
        """extract_speaker_embedding of several 24 kHz clips -> x-vectors fp32 [n][enc_dim] (device): clips of equal
        length share one ECAPA pass (rows of one batch; the reference calls it once per clip, W:434)."""
        ws = [self._dev_wav(w) for w in wavs]
        self._warn_range(ws)
        mels = [self.mel(w, check_range=False) for w in ws]
        out = torch.empty(len(ws), self.fc.N, dtype=torch.float32, device=self.dev)
        groups = {}
        for i, m in enumerate(mels):
            groups.setdefault(m.shape[0], []).append(i)
        for idx in groups.values():
            out[idx] = self.forward(torch.stack([mels[i] for i in idx]))
        return out
