"""bigdl_amd.transform — vision feature transformers (reference S/transform/**)."""
