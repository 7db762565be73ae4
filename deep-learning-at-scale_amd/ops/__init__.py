"""Device ops: the HIP kernel library bindings (``native``) and CPU reference math."""
