"""paddlebox_amd.runtime"""
