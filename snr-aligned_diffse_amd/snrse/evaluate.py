"""Evaluation driver: the loop of the reference's eval.py (eval.py:94-170) on the HIP path.

For every noisy file of <test_dir>/noisy (sorted): enhance with ScoreModel.enhance (PC or ODE
sampler), write <target_dir>/all/<name> (16-bit PCM, as soundfile's default for .wav), and
score it against <test_dir>/clean/<name>: PESQ (wide-band, 16 kHz) when the `pesq` package is
importable -- NaN otherwise, which is what the reference's try/except records on failure -- and
SI-SDR / SI-SIR / SI-SAR (utils.py:10-35, the columns the reference keeps commented out) from
the batched device kernel snrse_energy_ratios with n = y - x.  Results go to _results.csv and
_avg_results.txt ("mean ± std" over non-NaN values, utils.py:112-125).

Multi-GPU: files shard contiguously over ranks (snrse.dist.shard_range); the
per-file metric rows meet on every rank with one all_gather (RCCL over xGMI on the GPU box,
gloo in the CPU tests) and rank 0 writes the tables.

    python -m snrse.evaluate --test_dir DIR --ckpt CKPT --destination_folder OUT [--N 30 ...]
"""
from __future__ import annotations

import argparse
import os
from glob import glob
from os.path import join

import numpy as np
import torch

from . import audio, dist as sdist, ops

METRICS = ("pesq", "si_sdr", "si_sir", "si_sar")


def _pesq_fn():
    try:
        from pesq import pesq  # noqa: WPS433  (optional: absent in this image)
    except ImportError:
        return None
    return pesq


def print_mean_std(data, decimal=2):
    """utils.py:112-125: 'mean ± std' over the non-NaN values."""
    a = np.asarray(data, dtype=np.float64)
    a = a[~np.isnan(a)]
    if a.size == 0:
        return "nan ± nan"
    m, s = float(np.mean(a)), float(np.std(a))
    return f"{m:.3f} ± {s:.3f}" if decimal == 3 else f"{m:.2f} ± {s:.2f}"


def score_files(x_hat, x, y, sr=16000, pesq_fn=None):
    """One file's metric row (pesq, si_sdr, si_sir, si_sar); x_hat, x, y 1-D numpy float32."""
    L = min(len(x_hat), len(x), len(y))
    p = float("nan")
    if pesq_fn is not None:
        try:
            p = float(pesq_fn(sr, x[:L], x_hat[:L], "wb"))
        except Exception:  # the reference records NaN for any PESQ failure (eval.py:147-150)
            p = float("nan")
    dev = torch.device("cuda", torch.cuda.current_device())
    sig = torch.from_numpy(np.stack([x_hat[:L], x[:L], y[:L] - x[:L]]).astype(np.float32)).to(dev)
    er = ops.energy_ratios(sig[0:1], sig[1:2], sig[2:3])[0].cpu().numpy()
    return [p, float(er[0]), float(er[1]), float(er[2])]


def evaluate(model, test_dir, target_dir, sampler_type="pc", predictor="reverse_diffusion", corrector="ald",
             corrector_steps=1, snr=0.5, N=30, reverse_starting_point=1.0, force_N=0, atol=1e-5, rtol=1e-5,
             timestep_type="linear", correct_stepsize=False, oracle=False, rank=0, world=1, **enhance_kw):
    """-> dict with 'filename' and METRICS lists (all files, every rank)."""
    clean_dir, noisy_dir = join(test_dir, "clean"), join(test_dir, "noisy")
    os.makedirs(join(target_dir, "all"), exist_ok=True)
    if model.sde.__class__.__name__ == "OUVESDE":  # eval.py:105-108
        model.sde._T = reverse_starting_point
    else:
        model.sde.T = reverse_starting_point
    N = int(reverse_starting_point / (1 / N))
    if force_N:
        N = force_N
    clean_rms = noise_rms = None
    if oracle:  # per-file active RMS (eval.py:86-92 reads them from active_rms.txt)
        rows = [ln.split("\t") for ln in open(join(test_dir, "active_rms.txt")) if ln.strip()]
        clean_rms = [float(r[1]) for r in rows]
        noise_rms = [float(r[2]) for r in rows]
    files = sorted(glob(f"{noisy_dir}/*.wav"))
    a, b = sdist.shard_range(len(files), rank, world)
    pesq_fn = _pesq_fn()
    rows = []
    for i in range(a, b):
        name = os.path.basename(files[i])
        x, sr = audio.load(join(clean_dir, name))
        y, _ = audio.load(files[i])
        x_hat = model.enhance(x, y, sampler_type=sampler_type, predictor=predictor, corrector=corrector,
                              corrector_steps=corrector_steps, N=N, snr=snr, atol=atol, rtol=rtol,
                              timestep_type=timestep_type, correct_stepsize=correct_stepsize, oracle=oracle,
                              clean_rms=clean_rms[i] if oracle else 1, noise_rms=noise_rms[i] if oracle else 1,
                              **enhance_kw)
        audio.write_wav(join(target_dir, "all", name), x_hat, 16000, bits=16)
        rows.append(score_files(np.asarray(x_hat, np.float32), x[0].numpy(), y[0].numpy(), sr, pesq_fn))
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    allm = sdist.gather_metrics(rows if rows else np.zeros((0, len(METRICS))), len(files), rank, world,
                                dev if world > 1 and sdist_backend_is_nccl() else torch.device("cpu"))
    allm = allm.reshape(len(files), len(METRICS)).cpu().numpy()
    data = {"filename": [os.path.basename(f) for f in files]}
    for k, m in enumerate(METRICS):
        data[m] = [float(v) for v in allm[:, k]]
    if rank == 0:
        write_tables(data, target_dir)
    return data


def sdist_backend_is_nccl():
    import torch.distributed as tdist
    return tdist.is_available() and tdist.is_initialized() and tdist.get_backend() == "nccl"


def write_tables(data, target_dir):
    """_results.csv (one row per file) and _avg_results.txt (eval.py:159-170)."""
    with open(join(target_dir, "_results.csv"), "w") as f:
        f.write(",".join(["filename", *METRICS]) + "\n")
        for i, name in enumerate(data["filename"]):
            f.write(",".join([name] + [repr(float(data[m][i])) for m in METRICS]) + "\n")
    with open(join(target_dir, "_avg_results.txt"), "w") as f:
        f.write(f"PESQ: {print_mean_std(data['pesq'])} \n")
        f.write(f"SI-SDR: {print_mean_std(data['si_sdr'])} \n")
        f.write(f"SI-SIR: {print_mean_std(data['si_sir'])} \n")
        f.write(f"SI-SAR: {print_mean_std(data['si_sar'])} \n")


def main(argv=None):
    ap = argparse.ArgumentParser(description="eval.py on the MI355X path")
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
    ap.add_argument("--correct_stepsize", action="store_true")
    ap.add_argument("--oracle", action="store_true")
    a = ap.parse_args(argv)
    rank, world, _ = sdist.init_from_env()
    from sgmse.model import ScoreModel
    model = ScoreModel.load_from_checkpoint(a.ckpt, base_dir="", batch_size=16, num_workers=0, kwargs=dict(gpu=False))
    model.eval(no_ema=False)
    model.cuda()
    evaluate(model, a.test_dir, a.destination_folder, sampler_type=a.sampler_type, predictor=a.predictor,
             corrector=a.corrector, corrector_steps=a.corrector_steps, snr=a.snr, N=a.N,
             reverse_starting_point=a.reverse_starting_point, force_N=a.force_N, atol=a.atol, rtol=a.rtol,
             timestep_type=a.timestep_type, correct_stepsize=a.correct_stepsize, oracle=a.oracle, rank=rank,
             world=world)


if __name__ == "__main__":
    main()
