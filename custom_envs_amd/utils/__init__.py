"""Host-side utilities (logging, history) of the custom_envs surface."""
