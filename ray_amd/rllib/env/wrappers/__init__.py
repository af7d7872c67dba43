"""Environment wrappers (reference: rllib/env/wrappers/)."""
