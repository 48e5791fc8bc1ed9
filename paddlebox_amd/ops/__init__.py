"""paddlebox_amd.ops"""
