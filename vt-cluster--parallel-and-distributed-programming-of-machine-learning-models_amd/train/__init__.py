"""mift.train"""
