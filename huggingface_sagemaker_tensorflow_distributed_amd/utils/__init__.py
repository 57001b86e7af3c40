from .args import build_parser, hyperparameters_to_argv, parse_args, str2bool
from .env import dist_env, is_sagemaker_dp_enabled, sm_default
from .logging import LOG_FORMAT, setup_logging
from .results_io import write_eval_results, write_train_results

__all__ = [
    "build_parser", "parse_args", "str2bool", "hyperparameters_to_argv", "dist_env",
    "is_sagemaker_dp_enabled", "sm_default", "LOG_FORMAT", "setup_logging",
    "write_eval_results", "write_train_results",
]
