"""paddlebox_amd.metrics"""
