"""Command-line options with the reference's flag names and defaults (options.py:15-208).

Declared from one table so every flag of `MonodepthOptions` parses identically;
a few build-specific flags are appended at the end (marked "build:").
"""
from __future__ import annotations

import argparse
import os

_HERE = os.path.dirname(os.path.abspath(__file__))

# (flag, kwargs)
_FLAGS = [
    # paths
    ("--data_path", dict(type=str, default=os.path.join(_HERE, "kitti_data"), help="training data root")),
    ("--log_dir", dict(type=str, default=os.path.join(os.path.expanduser("~"), "tmp"), help="log directory")),
    # training
    ("--model_name", dict(type=str, default="mdp", help="folder name for the saved model")),
    ("--split", dict(type=str, default="eigen_zhou", choices=["eigen_zhou", "eigen_full", "odom", "benchmark"],
                     help="training split")),
    ("--num_layers", dict(type=int, default=18, choices=[18, 34, 50, 101, 152], help="ResNet depth")),
    ("--dataset", dict(type=str, default="kitti", choices=["kitti", "kitti_odom", "kitti_depth", "kitti_test"],
                       help="dataset")),
    ("--png", dict(action="store_true", help="train from png instead of jpg")),
    ("--height", dict(type=int, default=192, help="input height")),
    ("--width", dict(type=int, default=640, help="input width")),
    ("--disparity_smoothness", dict(type=float, default=1e-3, help="smoothness weight")),
    ("--scales", dict(nargs="+", type=int, default=[0, 1, 2, 3], help="loss scales")),
    ("--min_depth", dict(type=float, default=0.1, help="minimum depth")),
    ("--max_depth", dict(type=float, default=100.0, help="maximum depth")),
    ("--use_stereo", dict(action="store_true", help="add the stereo pair")),
    ("--frame_ids", dict(nargs="+", type=int, default=[0, -1, 1], help="frames to load")),
    # optimisation
    ("--batch_size", dict(type=int, default=12, help="batch size (per process)")),
    ("--learning_rate", dict(type=float, default=1e-4, help="Adam learning rate")),
    ("--num_epochs", dict(type=int, default=20, help="epochs")),
    ("--scheduler_step_size", dict(type=int, default=15, help="StepLR step")),
    # ablations
    ("--v1_multiscale", dict(action="store_true", help="monodepth v1 multiscale")),
    ("--avg_reprojection", dict(action="store_true", help="average instead of min reprojection")),
    ("--disable_automasking", dict(action="store_true", help="no auto-masking")),
    ("--predictive_mask", dict(action="store_true", help="predictive mask of Zhou et al.")),
    ("--no_ssim", dict(action="store_true", help="L1 only photometric loss")),
    ("--weights_init", dict(type=str, default="pretrained", choices=["pretrained", "scratch"],
                            help="encoder init")),
    ("--pose_model_input", dict(type=str, default="pairs", choices=["pairs", "all"], help="pose net input")),
    ("--pose_model_type", dict(type=str, default="separate_resnet",
                               choices=["posecnn", "separate_resnet", "shared"], help="pose network")),
    # system
    ("--no_cuda", dict(action="store_true", help="disable the GPU")),
    ("--num_workers", dict(type=int, default=12, help="data loader workers")),
    # loading
    ("--load_weights_folder", dict(type=str, help="checkpoint folder to load")),
    ("--models_to_load", dict(nargs="+", type=str, default=["encoder", "depth", "pose_encoder", "pose"],
                              help="models to load")),
    # logging
    ("--log_frequency", dict(type=int, default=250, help="batches between logs")),
    ("--save_frequency", dict(type=int, default=1, help="epochs between saves")),
    # evaluation
    ("--eval_stereo", dict(action="store_true", help="evaluate in stereo mode")),
    ("--eval_mono", dict(action="store_true", help="evaluate in mono mode")),
    ("--disable_median_scaling", dict(action="store_true", help="no median scaling")),
    ("--pred_depth_scale_factor", dict(type=float, default=1, help="prediction scale")),
    ("--ext_disp_to_eval", dict(type=str, help="external .npy disparities")),
    ("--eval_split", dict(type=str, default="eigen",
                          choices=["eigen", "eigen_benchmark", "benchmark", "odom_9", "odom_10"], help="eval split")),
    ("--save_pred_disps", dict(action="store_true", help="save predicted disparities")),
    ("--no_eval", dict(action="store_true", help="skip evaluation")),
    ("--eval_eigen_to_benchmark", dict(action="store_true", help="eigen npy evaluated on benchmark")),
    ("--eval_out_dir", dict(type=str, help="output folder for disparities")),
    ("--post_process", dict(action="store_true", help="flip post-processing")),
    # build-specific
    ("--materialize_images", dict(action="store_true",
                                  help="build: also materialise warped colours/samples/depth every step")),
    ("--noise_seed", dict(type=int, default=0, help="build: seed of the in-kernel tie-break noise")),
    ("--channels_last", dict(type=int, default=1,
                             help="build: 1 (default) NHWC activations/weights for the convolutions, 0 NCHW")),
    ("--hip_graph", dict(action="store_true", help="build: capture the whole training step in one hipGraph")),
    ("--pose_streams", dict(type=int, default=1,
                            help="build: 1 runs the pose network on its own HIP stream beside the depth network")),
    ("--amp", dict(type=str, default="none", choices=["none", "bf16"],
                   help="build: bf16 autocast for the networks (the photometric loss stays fp32)")),
    ("--grad_sync", dict(type=str, default="auto", choices=["auto", "ddp", "flat"],
                         help="build: gradient averaging for >1 GPU (auto: flat with --hip_graph, else ddp)")),
]


class MonodepthOptions:
    def __init__(self):
        self.parser = argparse.ArgumentParser(description="Monodepthv2 options (MI355X build)")
        for flag, kw in _FLAGS:
            self.parser.add_argument(flag, **kw)

    def parse(self, args=None):
        self.options = self.parser.parse_args(args)
        return self.options


def default_options(**overrides):
    """Parsed defaults with keyword overrides (for programmatic use and tests)."""
    opt = MonodepthOptions().parse([])
    for k, v in overrides.items():
        if not hasattr(opt, k):
            raise AttributeError(f"unknown option {k}")
        setattr(opt, k, v)
    return opt
