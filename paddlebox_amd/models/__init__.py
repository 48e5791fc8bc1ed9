"""paddlebox_amd.models"""
