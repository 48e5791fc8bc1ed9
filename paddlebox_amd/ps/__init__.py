"""paddlebox_amd.ps"""
