"""paddlebox_amd.parallel"""
