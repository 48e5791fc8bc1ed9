"""paddlebox_amd.fluid"""
