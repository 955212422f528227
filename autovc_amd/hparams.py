"""Hot-path slice of the reference's global config (autovc/utils/hparams.py:4-48).

Only the keys the Generator path and its neighbours (mel frontends, partial slices,
speaker encoder) read are restated: model dims, spectrogram settings, learn-loop defaults, Adam
settings and the dataloader batch size.  When this package is dropped into the reference tree
 the reference's own `AutoEncoderParams` dict can be passed in instead.
"""
from datetime import date

AutoEncoderParams = {
    "model_dir": "models/AutoVC",
    # hparams.py:6-14
    "spectrogram": {"sr": 22050, "n_mels": 80, "n_fft": 2048, "hop_length": 275, "window_length": 1100,
                    "fmin": 40, "mel_window_step": 12.5, "partial_utterance_n_frames": 400},
    "model": {"dim_neck": 32, "dim_emb": 256, "dim_pre": 512, "freq": 32},
    "learn": {
        "n_epochs": 1,
        "log_freq": 8,
        "save_freq": 16,
        "model_name": "model_" + date.today().strftime("%Y%m%d") + ".pt",
        "save_dir": "models/AutoVC",
        "ema_decay": 0.9999,
    },
    "optimizer": {
        "betas": (0.9, 0.999),
        "eps": 1e-8,
        "amsgrad": False,
        "lr": 1e-3,
        "weight_decay": 0.0,
        "lr_scheduler": "NoamScheduler",
        "n_warmup_steps": 256,
    },
    "dataloader": {"batch_size": 16},
}

# hparams.py:50-65 (inference keys of the speaker encoder)
SpeakerEncoderParams = {
    "model_dir": "models/SpeakerEncoder",
    "spectrogram": {"sr": 16000, "n_mels": 40, "mel_window_step": 10, "mel_window_length": 25,
                    "partial_utterance_n_frames": 160},
    "model": {"input_size": 40, "hidden_size": 256, "embedding_size": 256, "num_layers": 3,
              "batch_first": True},
    "learn": {"save_dir": "models/SpeakerEncoder"},
}

# hparams.py:92-115 (WaveRNNParams)
WaveRNNParams = {
    "model_dir": "models/WaveRNN",
    "model": {"hop_length": 275, "rnn_dims": 512, "res_out_dims": 128, "feat_dims": 80, "fc_dims": 512, "bits": 9,
              "upsample_factors": (5, 5, 11), "compute_dims": 128, "pad": 2, "res_blocks": 10, "mode": "MOL"},
    "generate": {"batched": True, "target": 11_000, "overlap": 550, "mu_law": False},
}
