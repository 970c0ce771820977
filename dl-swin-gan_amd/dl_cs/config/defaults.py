"""Default configuration values (same keys and values as the reference's
defaults.py:17-209, including its quirks: AUG_TRAIN.CROP_READOUT ends up 0,
CONV_BLOCK.COMPLEX defaults to True)."""

_C = {
    "VERSION": 1,
    "MODEL": {
        "DEVICE": "cuda", "NAME": "DLESPIRiT3D", "MODEL_TYPE": "RES", "WEIGHTS": "",
        "META_ARCHITECTURE": "dlespirit", "STRATEGY": "standard",
        "PARAMETERS": {
            "NUM_UNROLLS": 5, "NUM_RESBLOCKS": 2, "NUM_SWINBLOCKS": 2, "NUM_LAYERS": 4, "NUM_HEADS": 6,
            "RR": 16, "NUM_FEATURES": 256, "DROPOUT": 0.0, "NUM_EMAPS": 2, "NUM_COILS": 8,
            "NOISE_SCHED": "linear", "LEARN_SIGMA": False,
            "FIX_STEP_SIZE": False, "SHARE_WEIGHTS": False, "SLWIN_INIT": False, "GRAD_CHECKPOINT": False,
            "MODL": {"NUM_CG_STEPS": 10, "MU": 0.1, "FIX_PENALTY": False},
            "DSLR": {"NUM_BASIS": 8, "BLOCK_SIZE": 16, "OVERLAPPING": True, "NUM_CG_STEPS": 10},
            "WINDOW_SIZE": (4, 4), "NUM_HEAD": 4,
            "CONV_BLOCK": {"KERNEL_SIZE": (3,), "CIRCULAR_PAD": True, "ACTIVATION": "relu", "NORM": "none",
                           "SEPARABLE": True, "COMPLEX": True},
        },
        "RECON_LOSS": {"NAME": "complex_l1", "RENORMALIZE_DATA": True, "LOSS_WEIGHT": False},
    },
    "DATASET": {"TRAIN": (), "VAL": (), "TEST": ()},
    "DATALOADER": {"TRAIN_BATCH_SIZE": 1, "VAL_BATCH_SIZE": 1, "NUM_WORKERS": 4, "SUBSAMPLE": 1.0},
    "AUG_TRAIN": {
        "CROP_READOUT": 0, "ZPAD_PE": 0,
        "UNDERSAMPLE": {"NAME": "VDktMaskFunc", "ACCELERATIONS": (10, 15), "CALIBRATION_SIZE": 1,
                        "VD_POWER": 1.5, "PERTURB_FACTOR": 0.4, "ADHERE_FACTOR": 0.33,
                        "PARTIAL_KX": 0.25, "PARTIAL_KY": 0.0},
    },
    "AUG_VAL": {
        "UNDERSAMPLE": {"NAME": "VDktMaskFunc", "ACCELERATIONS": (10, 15), "CALIBRATION_SIZE": 1,
                        "VD_POWER": 1.5, "PERTURB_FACTOR": 0.4, "ADHERE_FACTOR": 0.33,
                        "PARTIAL_KX": 0.25, "PARTIAL_KY": 0.0},
    },
    "OPTIMIZER": {"NAME": "Adam", "MAX_EPOCHS": 1000, "GRAD_ACCUM_ITERS": 1, "GRAD_CLIP_VAL": 0.,
                  "ADAM": {"LR": 0.0001, "BETAS": (0.9, 0.999), "EPS": 1e-8, "WEIGHT_DECAY": 0.}},
    "LR_SCHEDULER": {"NAME": "StepLR", "STEP_SIZE": 1000, "GAMMA": 0.5},
    "EVAL": {"RUN_EVERY_N_EPOCHS": 1},
    "LOGGER": {"LOG_METRICS_EVERY_N_STEPS": 50, "LOG_IMAGES_EVERY_N_STEPS": 100,
               "LOG_PREDICTION_EVERY_N_STEPS": 500},
    # Swin-GAN (BASELINE config 3): build-defined, the reference names the run
    # (run_script.sh:29, :144-155) but ships no discriminator or config
    "GAN": {"ADV_WEIGHT": 0.01, "D_FEATURES": 160, "D_LR": 0.0001, "D_STEPS": 1},
    "OUTPUT_DIR": "", "DEVICE": -1, "SEED": 1, "CUDNN_BENCHMARK": False,
    "DESCRIPTION": {"BRIEF": "", "EXP_NAME": "", "TAGS": ()},
}
