"""paddlebox_amd.data"""
