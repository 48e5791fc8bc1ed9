"""paddlebox_amd.utils"""
