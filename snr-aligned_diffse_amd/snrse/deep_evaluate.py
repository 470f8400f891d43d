"""SNR-sweep evaluation: the loop of the reference's deep_eval.py (deep_eval.py:84-163) on the HIP path,
with the nine SNR variants of a file enhanced as ONE batch.

The reference re-mixes every test file at nine SNRs (deep_eval.py:108-118): with n = y - x,
y_S = x + n 10^(-S/20) for S = 0, 5, ..., 40, labelled S - 5 (-5 ... 35 dB), calls
ScoreModel.enhance once per variant (clean_rms = 1, noise_rms = 10^((5 - S)/20), used by the oracle
SNR branch), writes <target>/<label as %02d>/<name>, scores PESQ (wide-band; NaN when it fails or, here,
when `pesq` is not installed) and writes _results_deep.csv (filename, pesq_-5 ... pesq_35) and
_avg_results_deep.txt ("PESQ_<label>: mean ± std" with 3 decimals, utils.print_mean_std).

Here the nine variants share one length, so they are one batch of the device path, with the same
per-utterance arithmetic as the B=1 ScoreModel.enhance (model.py:702-839):
  * model_type 'bbed' + PC sampler: per-row max|y| normalisation, the fused STFT + transform, one
    batched ScoreModel.get_pc_sampler run (the sampler is batch-separable: every SDE scalar is per
    step, the network per utterance), iSTFT x max|y| per row;
  * 'sebridge_v3' + snr_conditioned 'true': snrse.enhance.SNRAlignedEnhancer (SNR from the estimator
    or, with --oracle, noise_rms / clean_rms; t_hat snapped per row);
  * anything else (the adaptive ODE sampler, whose step sizes depend on the whole state; the
    sebridge / sebridge_v2 one-step branches) runs the per-variant ScoreModel.enhance loop.
`si_sdr=True` adds si_sdr_<label> columns from snrse_energy_ratios (the reference keeps SI-SDR
commented out in this script, deep_eval.py:146-148).

Multi-GPU: files shard contiguously over ranks, rows meet with one all_gather.

    python -m snrse.deep_evaluate --test_dir DIR --ckpt CKPT --destination_folder OUT [--N 30 ...]
"""
from __future__ import annotations

import argparse
import os
from glob import glob
from os.path import join

import numpy as np
import torch

from . import audio, dist as sdist, ops
from .evaluate import _pesq_fn, print_mean_std, sdist_backend_is_nccl

SNRS = tuple(range(0, 41, 5))  # deep_eval.py:112
LABELS = tuple(s - 5 for s in SNRS)


def snr_variants(x, y):
    """deep_eval.py:108-118: x, y [L] -> (ys [9, L] float32, noise_rms [9]); clean_rms is 1."""
    x = np.asarray(x, np.float32).reshape(-1)
    y = np.asarray(y, np.float32).reshape(-1)
    n = y - x
    ys = np.stack([x + n * np.float32(10 ** (-s / 20)) for s in SNRS]).astype(np.float32)
    return ys, np.array([10 ** ((-s + 5) / 20) for s in SNRS], np.float64)


def _batched_kind(model, sampler_type):
    if model.snr_conditioned == "false" and model.model_type == "bbed" and sampler_type == "pc":
        return "pc"
    if model.snr_conditioned == "true" and model.model_type == "sebridge_v3":
        return "snr_aligned"
    return None


def enhance_variants(model, ys, noise_rms, clean_rms=1.0, sampler_type="pc", predictor="reverse_diffusion",
                     corrector="ald", corrector_steps=1, N=30, snr=0.5, oracle=False, batched=True,
                     noise_tape=None, **kwargs):
    """The nine model.enhance calls of one file (deep_eval.py:120-122).  ys [V, L] numpy f32 ->
    x_hat [V, L] numpy.  noise_tape(i) -> complex [V, F, T] injects the sampler's draws (parity runs;
    the per-variant path then receives row k of each draw)."""
    V, L = ys.shape
    kind = _batched_kind(model, sampler_type) if batched else None
    if kind is None:
        out = []
        for k in range(V):
            kw = dict(kwargs)
            if noise_tape is not None:
                kw["noise_tape"] = (lambda i, k=k: noise_tape(i)[k:k + 1].contiguous())
            out.append(model.enhance(torch.from_numpy(ys[k])[None], torch.from_numpy(ys[k])[None],
                                     sampler_type=sampler_type, predictor=predictor, corrector=corrector,
                                     corrector_steps=corrector_steps, N=N, snr=snr, oracle=oracle,
                                     clean_rms=clean_rms, noise_rms=float(noise_rms[k]), **kw))
        return np.stack(out)
    dev = torch.device("cuda", torch.cuda.current_device())
    yb = torch.from_numpy(np.ascontiguousarray(ys)).to(dev)
    mode = model.data_module.hip_mode()
    if kind == "pc":
        nf = ops.absmax(yb)  # per-row max|y| (model.py:726)
        Tp = L // 128 + 1
        Tp = Tp + (64 - Tp % 64) % 64
        Y = ops.stft(yb, 1.0, tpad=Tp, mode=mode, in_div=nf)
        sampler = model.get_pc_sampler(predictor, corrector, Y[:, None], N=N, corrector_steps=corrector_steps,
                                       snr=snr, noise_tape=noise_tape)
        sample, _ = sampler()
        xh = ops.istft(sample[:, 0].contiguous(), L, mode=mode, out_scale=nf)
        return xh.cpu().numpy()
    from .enhance import SNRAlignedEnhancer
    from sgmse.model import get_snr_model
    enh = SNRAlignedEnhancer(model.dnn.hip(dev), snr_fn=lambda spec: get_snr_model().estimate_from_spec(spec),
                             fixed_snr=float(model.fixed_snr), sigma_max=float(model.sigma_max),
                             transform=model.data_module.transform_type)
    est = np.asarray(noise_rms, np.float64) / float(clean_rms) if oracle else None  # model.py:722-724
    z = noise_tape(0) if noise_tape is not None else None
    xh, _ = enh(yb, est_snr=est, noise=z, seed=int(torch.randint(0, 2 ** 62, (1,)).item()))
    return xh.cpu().numpy()


def deep_evaluate(model, test_dir, target_dir, sampler_type="pc", predictor="reverse_diffusion", corrector="ald",
                  corrector_steps=1, snr=0.5, N=30, reverse_starting_point=1.0, force_N=0, atol=1e-5, rtol=1e-5,
                  timestep_type="linear", correct_stepsize=True, oracle=False, rank=0, world=1, batched=True,
                  si_sdr=False, noise_tapes=None, verbose=True):
    """-> dict: 'filename' and 'pesq_<label>' (+ 'si_sdr_<label>') lists over all files (every rank).
    noise_tapes(file_index) -> noise_tape for that file's batch (parity runs)."""
    clean_dir, noisy_dir = join(test_dir, "clean"), join(test_dir, "noisy")
    for lab in LABELS:
        os.makedirs(join(target_dir, "{0:02d}".format(lab)), exist_ok=True)
    if model.sde.__class__.__name__ == "OUVESDE":  # deep_eval.py:88-91
        model.sde._T = reverse_starting_point
    else:
        model.sde.T = reverse_starting_point
    N = int(reverse_starting_point / (1 / N))  # deep_eval.py:92-96
    if force_N:
        N = force_N
    files = sorted(glob("{}/*.wav".format(noisy_dir)))
    a, b = sdist.shard_range(len(files), rank, world)
    pesq_fn = _pesq_fn()
    ncol = len(LABELS) * (2 if si_sdr else 1)
    rows = []
    run = [0.0] * len(LABELS)
    for cnt, i in enumerate(range(a, b)):
        name = os.path.basename(files[i])
        x, sr = audio.load(join(clean_dir, name))
        y, _ = audio.load(files[i])
        x, y = x[0].numpy(), y[0].numpy()
        ys, noise_rms = snr_variants(x, y)
        xh = enhance_variants(model, ys, noise_rms, 1.0, sampler_type=sampler_type, predictor=predictor,
                              corrector=corrector, corrector_steps=corrector_steps, N=N, snr=snr, oracle=oracle,
                              batched=batched, noise_tape=None if noise_tapes is None else noise_tapes(i),
                              atol=atol, rtol=rtol, timestep_type=timestep_type, correct_stepsize=correct_stepsize)
        row = []
        for k, lab in enumerate(LABELS):
            audio.write_wav(join(target_dir, "{0:02d}".format(lab), name), xh[k], 16000, bits=16)
            p = float("nan")
            if pesq_fn is not None:
                try:
                    p = float(pesq_fn(sr, x, xh[k], "wb"))
                except Exception:  # deep_eval.py:134-137
                    p = float("nan")
            run[k] += p
            if verbose:
                print("{0} | {1:.3f}".format(lab, run[k] / (cnt + 1)), flush=True)
            row.append(p)
        if si_sdr:
            dev = torch.device("cuda", torch.cuda.current_device())
            Lm = min(xh.shape[1], len(x))
            xs = torch.from_numpy(np.ascontiguousarray(xh[:, :Lm], np.float32)).to(dev)
            cl = torch.from_numpy(np.repeat(x[None, :Lm], len(LABELS), 0)).to(dev)
            nz = torch.from_numpy(np.ascontiguousarray(ys[:, :Lm] - x[None, :Lm])).to(dev)
            row += [float(v) for v in ops.energy_ratios(xs, cl, nz)[:, 0].cpu().numpy()]
        rows.append(row)
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    allm = sdist.gather_metrics(rows if rows else np.zeros((0, ncol)), len(files), rank, world,
                                dev if world > 1 and sdist_backend_is_nccl() else torch.device("cpu"))
    allm = allm.reshape(len(files), ncol).cpu().numpy()
    data = {"filename": [os.path.basename(f) for f in files]}
    for k, lab in enumerate(LABELS):
        data[f"pesq_{lab}"] = [float(v) for v in allm[:, k]]
    if si_sdr:
        for k, lab in enumerate(LABELS):
            data[f"si_sdr_{lab}"] = [float(v) for v in allm[:, len(LABELS) + k]]
    if rank == 0:
        write_tables(data, target_dir)
    return data


def write_tables(data, target_dir):
    """_results_deep.csv (pandas to_csv(index=False) layout) and _avg_results_deep.txt (deep_eval.py:150-163)."""
    cols = [c for c in data if c != "filename"]
    with open(join(target_dir, "_results_deep.csv"), "w") as f:
        f.write(",".join(["filename", *cols]) + "\n")
        for i, name in enumerate(data["filename"]):
            f.write(",".join([name] + [repr(float(data[c][i])) for c in cols]) + "\n")
    with open(join(target_dir, "_avg_results_deep.txt"), "w") as f:
        for lab in LABELS:
            f.write("PESQ_{0}: {1} \n".format(lab, print_mean_std(data[f"pesq_{lab}"], decimal=3)))


def main(argv=None):
    ap = argparse.ArgumentParser(description="deep_eval.py (SNR sweep) on the MI355X path")
    ap.add_argument("--destination_folder", type=str, required=True)
    ap.add_argument("--test_dir", type=str, required=True)
    ap.add_argument("--ckpt", type=str, required=True)
    ap.add_argument("--sampler_type", type=str, choices=("pc", "ode"), default="pc")
    ap.add_argument("--predictor", type=str, default="reverse_diffusion")
    ap.add_argument("--reverse_starting_point", type=float, default=1.0)
    ap.add_argument("--force_N", type=int, default=0)
    ap.add_argument("--corrector", type=str, choices=("ald", "none"), default="ald")
    ap.add_argument("--corrector_steps", type=int, default=1)
    ap.add_argument("--snr", type=float, default=0.5)
    ap.add_argument("--N", type=int, default=30)
    ap.add_argument("--atol", type=float, default=1e-5)
    ap.add_argument("--rtol", type=float, default=1e-5)
    ap.add_argument("--timestep_type", type=str, default="linear")
    ap.add_argument("--correct_stepsize", dest="correct_stepsize", action="store_true")
    ap.add_argument("--no_correct_stepsize", dest="correct_stepsize", action="store_false")
    ap.add_argument("--modeltype", type=str, choices=["bbed", "sebridge", "sebridge_v2", "sebridge_v3"],
                    default="bbed")  # parsed and unused, as in deep_eval.py:45
    ap.add_argument("--oracle", action="store_true", help="SNR oracle (deep_eval.py's --oracle)")
    ap.add_argument("--per_variant", action="store_true", help="the reference's B=1 loop instead of one batch")
    ap.add_argument("--si_sdr", action="store_true")
    ap.set_defaults(correct_stepsize=True)
    a = ap.parse_args(argv)
    rank, world, _ = sdist.init_from_env()
    from sgmse.model import ScoreModel
    model = ScoreModel.load_from_checkpoint(a.ckpt, base_dir="", batch_size=16, num_workers=0, kwargs=dict(gpu=False))
    model.eval(no_ema=False)
    model.cuda()
    deep_evaluate(model, a.test_dir, a.destination_folder, sampler_type=a.sampler_type, predictor=a.predictor,
                  corrector=a.corrector, corrector_steps=a.corrector_steps, snr=a.snr, N=a.N,
                  reverse_starting_point=a.reverse_starting_point, force_N=a.force_N, atol=a.atol, rtol=a.rtol,
                  timestep_type=a.timestep_type, correct_stepsize=a.correct_stepsize, oracle=a.oracle,
                  rank=rank, world=world, batched=not a.per_variant, si_sdr=a.si_sdr)


if __name__ == "__main__":
    main()
