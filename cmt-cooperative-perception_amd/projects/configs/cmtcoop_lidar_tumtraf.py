# CMTCoop vehicle + infrastructure LiDAR only, TUMTraf shapes.
# Head block of the reference's CMTCoop_TUMTraf/lidar/coop/cmt_lidar_voxel0075_cbgs_a9coop_pretrained.py:167-297.
point_cloud_range = [-72.0, -72.0, -8, 72.0, 72.0, 0]
voxel_size = [0.1, 0.1, 0.2]
tumtraf_classes = ['CAR', 'TRAILER', 'TRUCK', 'VAN', 'PEDESTRIAN', 'BUS', 'BICYCLE']
grid_size = [1440, 1440, 40]
pts_voxel_layer = dict(num_point_features=5, max_num_points=10, voxel_size=voxel_size,
                       max_voxels=(120000, 160000), point_cloud_range=point_cloud_range)
head_type = 'CmtLidarHeadCoop'
transformer_type = 'CmtLidarTransformer'
final_kernel = 3
post_center_range = [-80, -80, -10.0, 80, 80, 10.0]
