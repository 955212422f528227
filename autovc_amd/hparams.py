"""Hot-path slice of the reference's global config (autovc/utils/hparams.py:4-48).

Only the keys the Generator path reads are restated: model dims, learn-loop defaults, Adam
settings and the dataloader batch size.  When this package is dropped into the reference tree
 the reference's own `AutoEncoderParams` dict can be passed in instead.
"""
from datetime import date

AutoEncoderParams = {
    "model_dir": "models/AutoVC",
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
