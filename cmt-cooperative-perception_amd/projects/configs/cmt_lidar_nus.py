# CMT-L (LiDAR only), nuScenes shapes -- BASELINE.json configs[1].
# Head block of the reference's CMT_Nuscenes/lidar/cmt_lidar_voxel0075_cbgs.py:161-288.
point_cloud_range = [-54.0, -54.0, -5.0, 54.0, 54.0, 3.0]
voxel_size = [0.075, 0.075, 0.2]
nus_classes = ['car', 'truck', 'construction_vehicle', 'bus', 'trailer', 'barrier', 'motorcycle', 'bicycle',
               'pedestrian', 'traffic_cone']
grid_size = [1440, 1440, 40]
pts_voxel_layer = dict(num_point_features=5, max_num_points=10, voxel_size=voxel_size,
                       max_voxels=(120000, 160000), point_cloud_range=point_cloud_range)
head_type = 'CmtLidarHead'
transformer_type = 'CmtLidarTransformer'
final_kernel = 3
post_center_range = [-61.2, -61.2, -10.0, 61.2, 61.2, 10.0]
