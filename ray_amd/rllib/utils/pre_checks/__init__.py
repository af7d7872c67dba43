from ray_amd.rllib.utils.pre_checks.env import check_env  # noqa: F401
