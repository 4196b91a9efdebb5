"""Namespace mirroring the reference's ``projects`` package (plugin_dir='projects/mmdet3d_plugin/')."""
