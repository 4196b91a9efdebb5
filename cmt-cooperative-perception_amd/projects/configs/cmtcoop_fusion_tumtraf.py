# CMTCoop vehicle + infrastructure camera+LiDAR, TUMTraf shapes -- BASELINE.json configs[3].
# Head block of the reference's CMTCoop_TUMTraf/fusion/coop/cmt_voxel0075_vov_1600x640_cbgs_a9coop_pretrained.py:270-360.
point_cloud_range = [-72.0, -72.0, -8, 72.0, 72.0, 0]
voxel_size = [0.1, 0.1, 0.2]
tumtraf_classes = ['CAR', 'TRAILER', 'TRUCK', 'VAN', 'PEDESTRIAN', 'BUS', 'BICYCLE']
grid_size = [1440, 1440, 40]
pts_voxel_layer = dict(num_point_features=5, max_num_points=10, voxel_size=voxel_size,
                       max_voxels=(120000, 160000), point_cloud_range=point_cloud_range)
head_type = 'CmtHeadCoop'
transformer_type = 'CmtTransformer'
final_kernel = 1
post_center_range = [-80, -80, -10.0, 80, 80, 10.0]
vehicle_cams = 1
infrastructure_cams = 3
final_dim = (640, 1600)
