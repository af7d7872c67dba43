"""``ray.tune.result`` (reference: python/ray/tune/result.py): the keys Tune writes into
every reported result dict (``trainable.py`` / ``tuner.py`` auto-fill them)."""

import os

DONE = "done"
SHOULD_CHECKPOINT = "should_checkpoint"
HOSTNAME = "hostname"
TRIAL_ID = "trial_id"
EXPERIMENT_TAG = "experiment_tag"
NODE_IP = "node_ip"
PID = "pid"
DEFAULT_METRIC = "_metric"
EPISODE_REWARD_MEAN = "episode_reward_mean"
MEAN_LOSS = "mean_loss"
MEAN_ACCURACY = "mean_accuracy"
EPISODES_THIS_ITER = "episodes_this_iter"
EPISODES_TOTAL = "episodes_total"
TIMESTEPS_THIS_ITER = "timesteps_this_iter"
TIMESTEPS_TOTAL = "timesteps_total"
TIME_THIS_ITER_S = "time_this_iter_s"
TIME_TOTAL_S = "time_total_s"
TRAINING_ITERATION = "training_iteration"
TIMESTAMP = "timestamp"
DATE = "date"
CONFIG = "config"

DEFAULT_EXPERIMENT_INFO_KEYS = ("trainable_name", EXPERIMENT_TAG, TRIAL_ID)
DEFAULT_RESULT_KEYS = (TRAINING_ITERATION, TIME_TOTAL_S, MEAN_ACCURACY, MEAN_LOSS)
AUTO_RESULT_KEYS = (TRAINING_ITERATION, TIME_TOTAL_S, EPISODES_TOTAL, TIMESTEPS_TOTAL,
                    DATE, TIMESTAMP, TIME_THIS_ITER_S, TRIAL_ID, EXPERIMENT_TAG,
                    HOSTNAME, NODE_IP, PID, DONE)
RESULT_DUPLICATE = "__duplicate__"
TRIAL_INFO = "__trial_info__"
STDOUT_FILE = "__stdout_file__"
STDERR_FILE = "__stderr_file__"
DEFAULT_RESULTS_DIR = os.environ.get("RAY_AMD_STORAGE", os.path.expanduser("~/ray_amd_results"))
DEFAULT_EXPERIMENT_NAME = "default"
EXPR_PROGRESS_FILE = "progress.csv"
EXPR_RESULT_FILE = "result.json"
EXPR_PARAM_FILE = "params.json"
CONFIG_PREFIX = "config"
