"""``ray.tune.constants`` (reference: python/ray/tune/constants.py): the environment
variables Tune reads."""

TUNE_ENV_VARS = {
    "RAY_AMD_STORAGE",          # default storage_path for runs (air/config.py RunConfig)
    "TUNE_MAX_PENDING_TRIALS_PG",
    "TUNE_RESULT_BUFFER_LENGTH",
    "TUNE_DISABLE_AUTO_CALLBACK_LOGGERS",
    "TUNE_GLOBAL_CHECKPOINT_S",
}
