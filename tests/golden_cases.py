"""Golden-fixture case table shared by make_golden.py and the tests."""

KWS_CASES = {
    # name: (hparams, batch kwargs)
    "L": (dict(n_layers=3, embedding_dim=128, learn_features=False, proj_mlp=False, frames_conv=False),
          dict(seed=11, K=6, ghost=(4,), plant=(1,), utt_len=1100)),
    "LE": (dict(n_layers=3, embedding_dim=128, learn_features=True, proj_mlp=True, frames_conv=False,
                proj_mlp_units=64),
           dict(seed=12, K=6, ghost=(4,), plant=(1,), utt_len=1500)),
    "LEF": (dict(n_layers=3, embedding_dim=128, learn_features=True, proj_mlp=True, frames_conv=True,
                 proj_mlp_units=64),
            dict(seed=13, K=8, ghost=(5,), plant=(1, 3), utt_len=1237)),
    "LEF_r18": (dict(n_layers=3, embedding_dim=128, learn_features=True, proj_mlp=True, frames_conv=True,
                     proj_mlp_units=64, resnet_version="resnet-18"),
                dict(seed=14, K=4, ghost=(), plant=(2,), utt_len=1500)),
}
THRESHOLDS = (0.3, 0.5)
