"""custom_envs.utils: the host-side helpers callers import."""
