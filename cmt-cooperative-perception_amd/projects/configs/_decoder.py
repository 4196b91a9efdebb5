# Shared pieces of the CMT head configs (mmcv dict style; loaded with
# projects.mmdet3d_plugin.config.load_config, never executed).
# Values follow the reference configs' pts_bbox_head blocks, e.g.
# projects/configs/CMT_Nuscenes/lidar/cmt_lidar_voxel0075_cbgs.py:197-257.
num_layers = 6
decoder = dict(
    type='PETRTransformerDecoder',
    return_intermediate=True,
    num_layers=num_layers,
    transformerlayers=dict(
        type='PETRTransformerDecoderLayer',
        with_cp=False,
        attn_cfgs=[
            dict(type='MultiheadAttention', embed_dims=256, num_heads=8, dropout=0.1),
            dict(type='PETRMultiheadFlashAttention', embed_dims=256, num_heads=8, dropout=0.1),
        ],
        ffn_cfgs=dict(type='FFN', embed_dims=256, feedforward_channels=1024, num_fcs=2, ffn_drop=0.,
                      act_cfg=dict(type='ReLU', inplace=True)),
        feedforward_channels=1024,
        operation_order=('self_attn', 'norm', 'cross_attn', 'norm', 'ffn', 'norm')),
)
common_heads = dict(center=(2, 2), height=(1, 2), dim=(3, 2), rot=(2, 2), vel=(2, 2))
