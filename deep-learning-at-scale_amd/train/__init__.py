"""wellflow.train"""
