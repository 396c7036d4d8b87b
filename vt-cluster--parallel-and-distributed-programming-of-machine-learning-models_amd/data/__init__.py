"""mift.data"""
